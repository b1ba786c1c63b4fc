#!/bin/bash
# in-DAG link model after the diag-first reorder: 2x4 la 1/2, chunk sizes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/ar; mkdir -p $D
for L in 25,50 10,150; do
  for la in 1 2; do
    timeout -k 10 200 python3 tools/r5/loopback_critpath.py --grid 2x4 --ranks 0,5 --lookahead $la --link $L > $D/lb_2x4_la${la}_$L.log 2>&1 || exit $?
    grep -h "job" $D/lb_2x4_la${la}_$L.log | sed "s/^/2x4 la=$la link=$L /"
  done
done
for ch in 2 8; do
  SLATE_AMD_POTRF_CHUNK=$ch timeout -k 10 200 python3 tools/r5/loopback_critpath.py --grid 2x4 --ranks 0,5 --link 25,50 > $D/lb_2x4_ch$ch.log 2>&1 || exit $?
  grep -h "job" $D/lb_2x4_ch$ch.log | sed "s/^/2x4 chunk=$ch link=25,50 /"
done
timeout -k 10 200 python3 tools/r5/loopback_critpath.py --grid 2x4 --ranks 0,5 > $D/lb_2x4_nolink.log 2>&1 || exit $?
grep -h "^| [0-9]" $D/lb_2x4_nolink.log
