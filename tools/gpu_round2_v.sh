#!/bin/bash
# potrf: trailing-update grouping x lookahead sweep (no reserved CUs)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sweep_v
for g in 2 4 6; do for la in 1 2; do
  SLATE_AMD_POTRF_GROUP=$g timeout -k 10 120 python -u bench.py --steps 4 --warmup 1 --check 0 --lookahead $la > gpurun_out/sweep_v/potrf_g${g}_la$la.log 2>&1 || exit 1
  echo "group=$g la=$la $(grep -o '"value": [0-9.]*' gpurun_out/sweep_v/potrf_g${g}_la$la.log)"
done; done
