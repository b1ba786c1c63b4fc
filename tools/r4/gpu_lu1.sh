#!/bin/bash
# LU RowMajor path: tests, then dgetrf bench RowMajor on/off
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${TAG:-lu1}; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_lu_rowmajor_gpu.py tests/test_nosync_gpu.py -x -v --timeout 120 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $D/pytest.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 200 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 > $D/bench_getrf_rm.log 2>&1 || { tail $D/bench_getrf_rm.log; exit 1; }
tail -1 $D/bench_getrf_rm.log
SLATE_AMD_LU_ROWMAJOR=0 timeout -k 10 200 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 > $D/bench_getrf_cm.log 2>&1 || { tail $D/bench_getrf_cm.log; exit 1; }
tail -1 $D/bench_getrf_cm.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=x timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run -- python3 -u bench.py --routine getrf --lookahead 2 --steps 1 --warmup 1 > $D/prof.log 2>&1 || { tail $D/prof.log; exit 1; }
echo prof ok
