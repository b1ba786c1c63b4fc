#!/bin/bash
# potrf loopback projections with / without step pairs at 2 and 4 GPUs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/ap; mkdir -p $D
for g in 1x2 2x1 2x2 4x1 1x4; do
  for pr in 1 0; do
    SLATE_AMD_POTRF_PAIR=$pr timeout -k 10 200 python3 tools/r5/loopback_critpath.py --grid $g --ranks 0 > $D/lb_${g}_p$pr.log 2>&1 || exit $?
    echo "$g pair=$pr: $(grep '^| 0' $D/lb_${g}_p$pr.log)"
  done
done
