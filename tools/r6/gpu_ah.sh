#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6/ah
for la in 1 2; do
 for inv in 2048 4096 8192; do
  SLATE_AMD_LU_INV_MIN=$inv timeout -k 10 300 python -u bench.py --impl native --routine getrf --steps 3 --warmup 1 --lookahead $la > gpurun_out/r6/ah/la${la}_inv$inv.json 2>/dev/null || exit 1
  echo "native la=$la inv_min=$inv $(python -c "import json;d=json.load(open('gpurun_out/r6/ah/la${la}_inv$inv.json'));print(d['value'], d['ms_per_step'])")"
 done
done
