#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for g in 1 2 3 4; do for la in 1 2; do
  v=$(SLATE_AMD_POTRF_GROUP=$g timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --lookahead $la 2>&1 | grep -o '"value": [0-9.]*\|"residual": [0-9.e-]*' | tr '\n' ' ') || exit 1
  echo "group=$g la=$la $v"
done; done
