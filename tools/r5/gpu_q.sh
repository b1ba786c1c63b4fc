#!/bin/bash
# kernel trace of the 2x4 loopback dpotrf, rank 0 (last step: the profiler may crash at teardown)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r5/q; mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/lb0 -o run -- python3 tools/r5/loopback_critpath.py --routine potrf --ranks 0 ${LBGRID:+--grid $LBGRID} ${LBLINK:+--link $LBLINK} ${LBLA:+--lookahead $LBLA} > $D/lb0.log 2>&1
echo "prof rc=$?"
