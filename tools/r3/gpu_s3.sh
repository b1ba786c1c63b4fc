#!/bin/bash
# LU base case v2 (unscaled-L elimination, one memset per panel): tests, panel latency, dgetrf bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${TAG:-s3}; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_native_gpu.py tests/test_nosync_gpu.py -x -q --timeout 120 --timeout-method thread -k "getrf or lu or gesv" > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/pytest.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 200 python -u tools/probe/lu_panel_time.py > $D/lu_panel_time.log 2>&1 || { tail $D/lu_panel_time.log; exit 1; }
cat $D/lu_panel_time.log
timeout -k 10 200 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 > $D/bench_getrf.log 2>&1 || { tail $D/bench_getrf.log; exit 1; }
tail -1 $D/bench_getrf.log
