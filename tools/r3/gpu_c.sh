#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3c
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3c/prof -o pmc -- python3 $GRAFT_REPO_ROOT/tools/probe/potrf_mc_prof.py 512 10 > $GRAFT_REPO_ROOT/gpurun_out/r3c/prof.log 2>&1 || { tail $GRAFT_REPO_ROOT/gpurun_out/r3c/prof.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/r3c/prof -name "*.csv" | head
