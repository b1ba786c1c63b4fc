#!/bin/bash
# stedc: 128-row leaves by default, two host round trips per merge: eig GPU tests, stedc timing, heev phases + bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${TAG:-s22}; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_eig_svd.py tests/test_dist_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $D/pytest.log
[ $rc -ne 0 ] && exit 1
PYTHONPATH=. timeout -k 10 200 python -u tools/probe/stedc_time.py > $D/stedc.log 2>&1 || { tail $D/stedc.log; exit 1; }
grep -v amdgpu.ids $D/stedc.log
timeout -k 10 300 python -u tools/heev_phases.py 16384 256 > $D/heev_phases.log 2>&1 || { tail $D/heev_phases.log; exit 1; }
cat $D/heev_phases.log
timeout -k 10 300 python -u bench.py --routine heev --n 16384 --nb 256 --steps 2 --warmup 1 > $D/bench_heev.log 2>&1 || { tail $D/bench_heev.log; exit 1; }
tail -1 $D/bench_heev.log | cut -c1-150
