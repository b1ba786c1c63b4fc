#!/bin/bash
# 8-GPU projections of dgetrf (lookahead 2) and dgemm, 2x4, in-DAG link model
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/az; mkdir -p $D
for L in 10,150 25,50; do
  timeout -k 10 300 python3 tools/r5/loopback_critpath.py --routine getrf --lookahead 2 --grid 2x4 --ranks 0,5 --steps 1 --link $L > $D/getrf_$L.log 2>&1 || { tail -20 $D/getrf_$L.log; exit 1; }
  grep -h "job" $D/getrf_$L.log | sed "s/^/getrf 2x4 la=2 link=$L /"
  timeout -k 10 300 python3 tools/r5/loopback_critpath.py --routine gemm --grid 2x4 --ranks 0,5 --steps 1 --link $L > $D/gemm_$L.log 2>&1 || { tail -20 $D/gemm_$L.log; exit 1; }
  grep -h "job" $D/gemm_$L.log | sed "s/^/gemm 2x4 link=$L /"
done
