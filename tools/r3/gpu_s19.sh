#!/bin/bash
# dgeqrf grouped bulk updates: QR GPU tests, bench group 1 / 2
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${TAG:-s19}; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_qr.py tests/test_nosync_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $D/pytest.log
[ $rc -ne 0 ] && exit 1
for g in 2 1; do
  SLATE_AMD_QR_GROUP=$g timeout -k 10 200 python -u bench.py --routine geqrf --rows 65536 --size 8192 --nb 256 --steps 3 --warmup 1 > $D/bench_geqrf_$g.log 2>&1 || { tail $D/bench_geqrf_$g.log; exit 1; }
  echo "group $g: $(tail -1 $D/bench_geqrf_$g.log | cut -c1-110) $(tail -1 $D/bench_geqrf_$g.log | grep -o '"residual[^,]*')"
done
