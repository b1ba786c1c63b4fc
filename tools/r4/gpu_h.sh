#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for cus in 32 16 0; do
  SLATE_AMD_PANEL_CUS=$cus timeout -k 10 300 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 > gpurun_out/getrf_cus$cus.log 2>&1; echo "cus=$cus rc=$?"
  tail -1 gpurun_out/getrf_cus$cus.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['residual'])"
done
