#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/aw; mkdir -p $D
for L in 10,150 25,50; do
  for ch in 16 32 64; do
    SLATE_AMD_POTRF_CHUNK=$ch timeout -k 10 200 python3 tools/r5/loopback_critpath.py --grid 2x4 --ranks 0,5 --link $L > $D/lb_$ch_$L.log 2>&1 || exit $?
    grep -h "job" $D/lb_$ch_$L.log | sed "s/^/2x4 ch=$ch link=$L /"
  done
  for ch in 4 16 64; do
    SLATE_AMD_POTRF_CHUNK=$ch timeout -k 10 200 python3 tools/r5/loopback_critpath.py --grid 2x2 --ranks 0 --link $L > $D/lb22_$ch_$L.log 2>&1 || exit $?
    grep -h "job" $D/lb22_$ch_$L.log | sed "s/^/2x2 ch=$ch link=$L /"
  done
done
