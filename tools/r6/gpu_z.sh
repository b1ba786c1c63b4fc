#!/bin/bash
# native heev n=16384: Q1 group sweep; Python dsyevd for comparison
set -o pipefail
mkdir -p gpurun_out/r6/z
for g in 4 8 16; do
  SLATE_AMD_UNMTR_HE2HB_GROUP=$g timeout -k 10 300 slate_amd/bench_native heev 16384 256 1 1 1 1 2 0 > gpurun_out/r6/z/g$g.log 2>&1 || exit $?
  echo "group $g: $(grep RESULT gpurun_out/r6/z/g$g.log)"
done
timeout -k 10 600 python -u bench.py --routine heev --size 16384 --nb 256 --steps 2 --warmup 1 > gpurun_out/r6/z/py_heev.log 2>&1
rc=$?
tail -2 gpurun_out/r6/z/py_heev.log
exit $rc
