#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/bc; mkdir -p $D
for L in 10,150 25,50; do
  for la in 1 2 3; do
    timeout -k 10 200 python3 tools/r5/loopback_critpath.py --grid 2x4 --ranks 0,5 --lookahead $la --link $L > $D/lb_${la}_$L.log 2>&1 || exit $?
    grep -h "job" $D/lb_${la}_$L.log | sed "s/^/2x4 la=$la link=$L /"
  done
done
for la in 1 2; do
  timeout -k 10 200 python3 tools/r5/loopback_critpath.py --grid 2x2 --ranks 0 --lookahead $la --link 10,150 > $D/lb22_${la}.log 2>&1 || exit $?
  grep -h "job" $D/lb22_${la}.log | sed "s/^/2x2 la=$la link=10,150 /"
done
