#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && export PYTHONPATH="$GRAFT_REPO_ROOT"
O=gpurun_out/r3i
mkdir -p $O
timeout -k 10 120 python -u tools/probe/graph_probe2.py C > $O/graph_probe2_C.log 2>&1
echo "rc=$?"; grep -v amdgpu.ids $O/graph_probe2_C.log | grep -v "^  File\|^Extension\|^$\|Current thread" | tail -4
timeout -k 10 180 python -u tools/probe/graph_probe.py > $O/graph_probe.log 2>&1
echo "rc=$?"; grep -v amdgpu.ids $O/graph_probe.log | tail -8
exit 0
