#!/bin/bash
# hb2st sweep-resident window: eig GPU tests; chase timing with / without reuse; heev bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${TAG:-s17}; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_eig_svd.py -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $D/pytest.log
[ $rc -ne 0 ] && exit 1
for r in 1 0; do
  SLATE_AMD_HB2ST_REUSE=$r HB2ST_PROBE_NOHOST=1 timeout -k 10 120 python -u tools/probe/hb2st_time.py 16384 64 > $D/hb2st_$r.log 2>&1 || { tail -3 $D/hb2st_$r.log; exit 1; }
  echo "reuse $r: $(grep device $D/hb2st_$r.log) | $(grep phases $D/hb2st_$r.log | cut -c1-90)"
done
timeout -k 10 300 python -u bench.py --routine heev --n 16384 --nb 256 --steps 2 --warmup 1 > $D/bench_heev.log 2>&1 || { tail $D/bench_heev.log; exit 1; }
tail -1 $D/bench_heev.log | cut -c1-150
