#!/bin/bash
# dgeqrf kernel profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${TAG:-s15}; mkdir -p $D
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof_geqrf -o run -- python3 $GRAFT_REPO_ROOT/bench.py --routine geqrf --rows 65536 --size 8192 --nb 256 --steps 1 --warmup 1 --check 0 > $GRAFT_REPO_ROOT/$D/prof_geqrf.log 2>&1
echo "prof rc=$?"; grep metric $GRAFT_REPO_ROOT/$D/prof_geqrf.log | cut -c1-150
