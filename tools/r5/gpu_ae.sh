#!/bin/bash
# masked trailing GEMM of the 2x4 dpotrf in isolation: block order / group size
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for cfg in "0 8" "1 8" "3 8" "3 2" "3 4" "0 1" "3 16"; do
  set -- $cfg
  echo "remap $1 group $2:"; SLATE_AMD_GEMM_MASK_REMAP=$1 SLATE_AMD_GEMM_GROUP=$2 timeout -k 10 120 python3 tools/r5/masked_gemm_probe.py 2>&1 | grep -E "TF/s" || exit 1
done
