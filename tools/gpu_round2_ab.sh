#!/bin/bash
# getrf: one row per thread below a panel-height threshold (tail), two above
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sweep_ab
for th in 0 8192 16384 24576; do
  SLATE_AMD_LU_RPT1_ROWS=$th timeout -k 10 150 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 --check 0 > gpurun_out/sweep_ab/getrf_t$th.log 2>&1 || exit 1
  echo "rpt1_rows=$th $(grep -o '"value": [0-9.]*' gpurun_out/sweep_ab/getrf_t$th.log)"
done
