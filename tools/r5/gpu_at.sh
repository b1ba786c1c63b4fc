#!/bin/bash
# 2x4 potrf, in-DAG link model: CUs reserved for the panel / diag streams
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/at; mkdir -p $D
for L in 10,150 25,50; do
  for cus in 0 16 32 64; do
    SLATE_AMD_PANEL_CUS=$cus timeout -k 10 200 python3 tools/r5/loopback_critpath.py --grid 2x4 --ranks 0,5 --link $L > $D/lb_${cus}_$L.log 2>&1 || exit $?
    grep -h "job" $D/lb_${cus}_$L.log | sed "s/^/2x4 cus=$cus link=$L /"
  done
done
for cus in 0 32; do
  SLATE_AMD_PANEL_CUS=$cus timeout -k 10 200 python3 tools/r5/loopback_critpath.py --grid 2x2 --ranks 0 --link 10,150 > $D/lb22_${cus}.log 2>&1 || exit $?
  grep -h "job" $D/lb22_${cus}.log | sed "s/^/2x2 cus=$cus link=10,150 /"
done
