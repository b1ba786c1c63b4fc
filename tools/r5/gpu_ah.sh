#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r5/ah; mkdir -p $D
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $D/pr -o run -- python3 tools/r5/masked_gemm_probe.py > $D/pr.log 2>&1
echo "rc=$?"
