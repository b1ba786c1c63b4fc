#!/bin/bash
# 8-GPU projection of dgemm n = 32768 (SUMMA, 2x4) under the in-DAG link model
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/ba; mkdir -p $D
for L in 10,150 25,50; do
  timeout -k 10 300 python3 tools/r5/loopback_critpath.py --routine gemm --grid 2x4 --ranks 0,5 --steps 1 --link $L > $D/gemm_$L.log 2>&1 || { tail -20 $D/gemm_$L.log; exit 1; }
  grep -h "job" $D/gemm_$L.log | sed "s/^/gemm 2x4 link=$L /"
done
