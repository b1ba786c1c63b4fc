#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${TAG:-b}; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_lu_rowmajor_gpu.py tests/test_dist_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/pytest.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 200 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 > $D/bench_getrf.log 2>&1 || { tail $D/bench_getrf.log; exit 1; }
tail -1 $D/bench_getrf.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run -- python3 -u bench.py --routine getrf --lookahead 2 --steps 1 --warmup 1 > $D/prof.log 2>&1
echo "prof rc=$?"
