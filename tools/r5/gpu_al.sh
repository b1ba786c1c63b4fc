#!/bin/bash
# loopback dpotrf projection for the 2- and 4-GPU grid shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/al; mkdir -p $D
for g in 1x2 2x1 2x2 4x1 1x4; do
  P=${g%x*}; Q=${g#*x}; last=$((P*Q-1))
  timeout -k 10 300 python -u tools/r5/loopback_critpath.py --routine potrf --grid $g --ranks 0,$last > $D/potrf_$g.log 2>&1 || { tail -5 $D/potrf_$g.log; exit 1; }
  echo "$g: $(grep 'Job projection' $D/potrf_$g.log)"
done
