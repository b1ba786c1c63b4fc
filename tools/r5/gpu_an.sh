#!/bin/bash
# stair mapping rewrite: kernel tests + per-step probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/an; mkdir -p $D
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "trimask or stair or gemm" > $D/kt.log 2>&1 || { tail -30 $D/kt.log; exit 1; }
tail -3 $D/kt.log
for g in 1x1 1x2 2x1 2x2 2x4; do
  timeout -k 10 120 python3 tools/r5/stair_probe.py --grid $g >> $D/probe.log 2>&1 || exit $?
done
SLATE_AMD_GEMM_TRI=0 timeout -k 10 120 python3 tools/r5/stair_probe.py --grid 1x1 >> $D/probe.log 2>&1
cat $D/probe.log
