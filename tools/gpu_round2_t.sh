#!/bin/bash
# tpqrt kernels + multi-rank rehearsal (TSQR tree by tpqrt), then potrf/getrf kernel traces
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_tpqrt.py tests/test_eig_svd.py tests/test_dist_gpu.py tests/test_qr.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_t.log 2>&1 || { tail -40 gpurun_out/pytest_t.log; exit 1; }
tail -2 gpurun_out/pytest_t.log
bash tools/gpu_prof_csv.sh potrf --steps 1 --warmup 1 && bash tools/gpu_prof_csv.sh getrf --routine getrf --lookahead 2 --steps 1 --warmup 1
