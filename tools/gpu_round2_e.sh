#!/bin/bash
# Round-2: distributed eigensolver on the GPU + heev timings.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py tests/test_eig_svd.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_eig_gpu.log 2>&1
rc=$?; echo "eig gpu tests rc=$rc"; tail -4 gpurun_out/pytest_eig_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/probe/heev_breakdown.py 8192 256 2>&1 | grep -v amdgpu.ids || exit 1
SLATE_AMD_EIG_DIST=1 timeout -k 10 300 python -u tools/probe/heev_breakdown.py 8192 256 2>&1 | grep -v amdgpu.ids || exit 1
