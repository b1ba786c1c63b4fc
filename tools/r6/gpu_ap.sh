#!/bin/bash
# native heev n=16384: chase workgroup count sweep (default = nt0/3 + 15 = 100)
set -o pipefail
mkdir -p gpurun_out/r6/ap
for w in 0 72 86 128 170 256; do
  SLATE_AMD_HB2ST_NWG=$w timeout -k 10 200 slate_amd/bench_native heev 16384 256 1 1 1 1 2 0 > gpurun_out/r6/ap/nwg$w.log 2>&1 || { tail -5 gpurun_out/r6/ap/nwg$w.log; exit 1; }
  echo "nwg=$w $(grep RESULT gpurun_out/r6/ap/nwg$w.log)" | tee -a gpurun_out/r6/ap/sweep.txt
done
