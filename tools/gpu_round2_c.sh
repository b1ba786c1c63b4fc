#!/bin/bash
# Round-2: persistent-LU failure handling + distributed LU on the GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "getrf" --timeout 120 --timeout-method thread > gpurun_out/pytest_getrf.log 2>&1
rc=$?; echo "getrf kernel tests rc=$rc"; tail -4 gpurun_out/pytest_getrf.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u tools/probe/lu_grid_gpu.py > gpurun_out/lu_grid.log 2>&1
rc=$?; echo "probe rc=$rc"; grep "^grid" gpurun_out/lu_grid.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_dist_gpu.log 2>&1
rc=$?; echo "dist gpu tests rc=$rc"; tail -4 gpurun_out/pytest_dist_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 > gpurun_out/bench_getrf.log 2>&1 || exit 1
tail -1 gpurun_out/bench_getrf.log
