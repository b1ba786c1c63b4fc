#!/bin/bash
# LU panel latency per height + kernel trace of one m=8192 panel
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s2
timeout -k 10 200 python -u tools/probe/lu_panel_time.py > gpurun_out/s2/lu_panel_time.log 2>&1 || { tail gpurun_out/s2/lu_panel_time.log; exit 1; }
cat gpurun_out/s2/lu_panel_time.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/s2/prof8192 -o run -- python3 $GRAFT_REPO_ROOT/tools/probe/lu_panel_once.py 8192 > $GRAFT_REPO_ROOT/gpurun_out/s2/prof8192.log 2>&1 || { tail $GRAFT_REPO_ROOT/gpurun_out/s2/prof8192.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/s2/prof8192 -name "*stats*" | head
