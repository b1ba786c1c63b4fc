#!/bin/bash
# Round-2: distributed LU machinery on the GPU + getrf bench (pp and CALU).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_dist_gpu.log 2>&1
rc=$?; echo "dist gpu tests rc=$rc"; tail -5 gpurun_out/pytest_dist_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 > gpurun_out/bench_getrf.log 2>&1 || exit 1
tail -1 gpurun_out/bench_getrf.log
