#!/bin/bash
# Python dsyevd n=16384: Q1 group size 4 (default) vs 8
set -o pipefail
mkdir -p gpurun_out/r6/ar
for g in 4 8; do
  SLATE_AMD_UNMTR_HE2HB_GROUP=$g timeout -k 10 300 python bench.py --routine heev --size 16384 --nb 256 --steps 3 --warmup 1 > gpurun_out/r6/ar/g$g.json 2> gpurun_out/r6/ar/g$g.err || { tail -5 gpurun_out/r6/ar/g$g.err; exit 1; }
  echo "G=$g $(cat gpurun_out/r6/ar/g$g.json)" | cut -c1-160
done
