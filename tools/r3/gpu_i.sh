#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && export PYTHONPATH="$GRAFT_REPO_ROOT"
O=gpurun_out/r3i
mkdir -p $O
true
rc=0
[ $rc -ne 0 ] && exit 1
timeout -k 10 200 python -u tools/probe/graph_time.py > $O/graph_time.log 2>&1
echo "graph_time rc=$?"; grep -v amdgpu.ids $O/graph_time.log | tail -6
exit 0
