#!/bin/bash
# loopback dpotrf projection over the 8-GPU grid shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/s; mkdir -p $D
for g in 2x4 4x2 1x8 8x1; do
  timeout -k 10 300 python -u tools/r5/loopback_critpath.py --routine potrf --grid $g --ranks 0,3,7 > $D/potrf_$g.log 2>&1 || { tail -5 $D/potrf_$g.log; exit 1; }
  echo "$g: $(grep 'Job projection' $D/potrf_$g.log)"
  grep -E '^\| [037] ' $D/potrf_$g.log
done
