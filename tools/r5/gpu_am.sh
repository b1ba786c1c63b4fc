#!/bin/bash
# masked trailing-update efficiency per step, 1x1 vs 1x2 vs 2x2 vs 2x4
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/am; mkdir -p $D
for g in 1x1 1x2 2x1 2x2 2x4; do
  timeout -k 10 120 python3 tools/r5/stair_probe.py --grid $g >> $D/probe.log 2>&1 || exit $?
done
for g in 1x1 1x2; do
  timeout -k 10 120 python3 tools/r5/stair_probe.py --grid $g --K 1024 >> $D/probe.log 2>&1 || exit $?
done
SLATE_AMD_GEMM_MASK_REMAP=0 timeout -k 10 120 python3 tools/r5/stair_probe.py --grid 1x2 >> $D/probe.log 2>&1
cat $D/probe.log
