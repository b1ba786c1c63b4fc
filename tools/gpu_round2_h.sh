#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "trsm or potrf" --timeout 120 --timeout-method thread > gpurun_out/pytest_k.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -2 gpurun_out/pytest_k.log; [ $rc -eq 0 ] || exit 1
for r in potrf getrf; do timeout -k 10 200 python -u bench.py --routine $r --steps 5 --warmup 2 2>&1 | grep -o '"value": [0-9.]*' || exit 1; done
timeout -k 10 200 python -u bench.py --routine geqrf --m 65536 --n 8192 --nb 256 --steps 3 --warmup 1 2>&1 | grep -o '"value": [0-9.]*' || exit 1
