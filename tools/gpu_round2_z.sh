#!/bin/bash
# getrf: rows per thread 2, reserved panel CUs sweep (repeat for noise)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sweep_z
for cfg in "2 32 2" "2 24 2" "2 16 2" "2 32 1" "2 48 2" "2 32 2" "1 64 2"; do
  set -- $cfg
  SLATE_AMD_LU_RPT=$1 SLATE_AMD_PANEL_CUS=$2 timeout -k 10 150 python -u bench.py --routine getrf --lookahead $3 --steps 3 --warmup 1 --check 0 > gpurun_out/sweep_z/getrf_r$1_c$2_la$3.log 2>&1 || exit 1
  echo "rpt=$1 cus=$2 la=$3 $(grep -o '"value": [0-9.]*' gpurun_out/sweep_z/getrf_r$1_c$2_la$3.log)"
done
