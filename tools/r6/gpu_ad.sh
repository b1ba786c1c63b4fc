#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6/ad
for keep in 0 1; do
  SLATE_AMD_NATIVE_KEEP_RESERVATION=$keep timeout -k 10 300 python -u bench.py --impl native --routine getrf --steps 3 --warmup 1 > gpurun_out/r6/ad/k$keep.json 2>/dev/null || exit 1
  echo "keep=$keep $(python -c "import json;d=json.load(open('gpurun_out/r6/ad/k$keep.json'));print(d['value'], d['ms_per_step'])")"
done
SLATE_AMD_NATIVE_KEEP_RESERVATION=1 timeout -k 10 300 python -u bench.py --impl native --steps 3 --warmup 1 > gpurun_out/r6/ad/potrf_k1.json 2>/dev/null || exit 1
echo "potrf keep=1 $(python -c "import json;d=json.load(open('gpurun_out/r6/ad/potrf_k1.json'));print(d['value'], d['ms_per_step'])")"
