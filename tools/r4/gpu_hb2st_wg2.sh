#!/bin/bash
# dsyevd n = 16384, chase workgroups 72..136, 2 timed steps each
mkdir -p gpurun_out/r4
for wg in 136 100 84 120 100 136; do
  SLATE_AMD_HB2ST_WG=$wg timeout -k 10 120 python bench.py --routine heev --n 16384 --steps 2 --warmup 1 > gpurun_out/r4/hb2st_wg2_$wg.log 2>&1 || exit $?
  echo "wg=$wg $(grep -o '"value": [0-9.]*' gpurun_out/r4/hb2st_wg2_$wg.log)"
done
