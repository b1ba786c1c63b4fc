#!/bin/bash
# 4-GPU and 2-GPU grid shapes for potrf under the in-DAG link model (current code)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/bf; mkdir -p $D
for L in 10,150 25,50; do
  for g in 2x2 1x4 4x1 1x2 2x1; do
    timeout -k 10 200 python3 tools/r5/loopback_critpath.py --grid $g --ranks 0 --link $L > $D/lb_${g}_$L.log 2>&1 || exit $?
    grep -h "job" $D/lb_${g}_$L.log | sed "s/^/$g link=$L /"
  done
done
