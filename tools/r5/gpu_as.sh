#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/as2; mkdir -p $D
for ks in 1 2 4; do
  SLATE_AMD_TRSM_KS=$ks timeout -k 10 120 python3 tools/r5/trsm_probe.py 2>&1 | grep -v amdgpu | sed "s/^/ks=$ks /" >> $D/trsm.log || { cat $D/trsm.log; exit 1; }
done
cat $D/trsm.log
