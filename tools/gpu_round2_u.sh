#!/bin/bash
# potrf: reserved panel CUs x trailing-update grouping sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sweep_u
for cus in 0 2 4 8 16; do
  SLATE_AMD_PANEL_CUS=$cus timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --check 0 > gpurun_out/sweep_u/potrf_c$cus.log 2>&1 || exit 1
  echo "cus=$cus $(grep -o '"value": [0-9.]*' gpurun_out/sweep_u/potrf_c$cus.log)"
done
for g in 3 4; do
  SLATE_AMD_PANEL_CUS=8 SLATE_AMD_POTRF_GROUP=$g timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --check 0 > gpurun_out/sweep_u/potrf_g$g.log 2>&1 || exit 1
  echo "cus=8 group=$g $(grep -o '"value": [0-9.]*' gpurun_out/sweep_u/potrf_g$g.log)"
done
for cus in 0 8 16; do
  SLATE_AMD_PANEL_CUS=$cus timeout -k 10 120 python -u bench.py --routine getrf --lookahead 2 --steps 2 --warmup 1 --check 0 > gpurun_out/sweep_u/getrf_c$cus.log 2>&1 || exit 1
  echo "getrf cus=$cus $(grep -o '"value": [0-9.]*' gpurun_out/sweep_u/getrf_c$cus.log)"
done
