#!/bin/bash
# 2x4 dpotrf projections under the per-link model: ring broadcasts (every
# link carries the message) vs the direct scatter + all-gather row broadcast
# (SLATE_AMD_BCAST_SA=1: 2 B / q per link)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6/p; mkdir -p $D
for L in 25,50 10,150 25,76; do
  for sa in 0 1; do
    SLATE_AMD_BCAST_SA=$sa timeout -k 10 240 python3 tools/r5/loopback_critpath.py --grid 2x4 --ranks 0,5 --link $L > $D/lb_sa${sa}_$L.log 2>&1 || { tail -20 $D/lb_sa${sa}_$L.log; exit 1; }
    grep -h "job" $D/lb_sa${sa}_$L.log | sed "s/^/2x4 sa=$sa link=$L /"
  done
done
