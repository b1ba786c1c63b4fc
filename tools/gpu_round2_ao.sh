#!/bin/bash
# quad-lane compute in the tb2bd task: SVD GPU tests + tb2bd timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_eig_svd.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ao.log 2>&1 || { tail -30 gpurun_out/pytest_ao.log; exit 1; }
tail -1 gpurun_out/pytest_ao.log
timeout -k 10 300 python -u tools/probe/tb2bd_time.py 8192 64
