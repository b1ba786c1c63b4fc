#!/bin/bash
# explicit V^H in both geqrf paths: GPU QR + multi-rank rehearsal tests with V^H forced on
set -o pipefail
cd "$GRAFT_REPO_ROOT"
SLATE_AMD_QR_VH_ROWS=1 timeout -k 10 400 python -u -m pytest tests/test_qr.py tests/test_dist_gpu.py tests/test_tpqrt.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ai.log 2>&1 || { tail -30 gpurun_out/pytest_ai.log; exit 1; }
tail -1 gpurun_out/pytest_ai.log
