#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6/af
for sh in 0 1 2 3; do
  SLATE_AMD_QUEUE_SHIFT=$sh timeout -k 10 300 python -u bench.py --routine getrf --steps 3 --warmup 1 > gpurun_out/r6/af/getrf_s$sh.json 2>/dev/null || exit 1
  echo "getrf shift=$sh $(python -c "import json;d=json.load(open('gpurun_out/r6/af/getrf_s$sh.json'));print(d['value'], d['ms_per_step'])")"
done
for sh in 0 1 2 3; do
  SLATE_AMD_QUEUE_SHIFT=$sh timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/r6/af/potrf_s$sh.json 2>/dev/null || exit 1
  echo "potrf shift=$sh $(python -c "import json;d=json.load(open('gpurun_out/r6/af/potrf_s$sh.json'));print(d['value'], d['ms_per_step'])")"
done
