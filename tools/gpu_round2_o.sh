#!/bin/bash
# lookahead sweeps (geqrf, potrf) and dgemm at the BASELINE size
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for la in 1 2 3; do
  v=$(timeout -k 10 200 python -u bench.py --routine geqrf --m 65536 --n 8192 --nb 256 --lookahead $la --steps 3 --warmup 1 2>&1 | grep -o '"value": [0-9.]*\|"residual": [0-9.e-]*' | tr '\n' ' ') || exit 1
  echo "geqrf la=$la $v"
done
for la in 1 2; do
  v=$(timeout -k 10 200 python -u bench.py --lookahead $la --steps 5 --warmup 2 2>&1 | grep -o '"value": [0-9.]*\|"residual": [0-9.e-]*' | tr '\n' ' ') || exit 1
  echo "potrf la=$la $v"
done
v=$(timeout -k 10 200 python -u bench.py --routine gemm --n 32768 --steps 2 --warmup 1 2>&1 | grep -o '"value": [0-9.]*' | tr '\n' ' ') || exit 1
echo "gemm n=32768 $v"
