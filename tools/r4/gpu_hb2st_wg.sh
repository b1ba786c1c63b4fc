#!/bin/bash
# dsyevd n = 16384 with different chase workgroup counts (default: min(CUs, tasks/2 + 8) = 136)
mkdir -p gpurun_out/r4
for wg in 136 100 176 220 256; do
  SLATE_AMD_HB2ST_WG=$wg timeout -k 10 120 python bench.py --routine heev --n 16384 --steps 1 --warmup 1 > gpurun_out/r4/hb2st_wg_$wg.log 2>&1 || exit $?
  echo "wg=$wg $(grep -o '"value": [0-9.]*' gpurun_out/r4/hb2st_wg_$wg.log)"
done
