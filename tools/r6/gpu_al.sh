#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6/al
for n in 4096 16384; do
  timeout -k 10 300 slate_amd/bench_native heev $n 256 1 1 1 1 1 1 > gpurun_out/r6/al/heev$n.log 2>&1 || { cat gpurun_out/r6/al/heev$n.log; exit 1; }
  echo "n=$n $(grep RESULT gpurun_out/r6/al/heev$n.log)"
done
SLATE_AMD_UNMTR_HE2HB_GROUP=8 timeout -k 10 300 slate_amd/bench_native heev 16384 256 1 1 1 1 2 0 > gpurun_out/r6/al/g8.log 2>&1 && echo "g8 $(grep RESULT gpurun_out/r6/al/g8.log)"
