#!/bin/bash
# native heev: Q1 merges / Q2 T factors on the side stream (overlap) vs serial
set -o pipefail
mkdir -p gpurun_out/r6/am
for n in 4096 16384; do
  timeout -k 10 300 slate_amd/bench_native heev $n 256 1 1 1 1 2 1 > gpurun_out/r6/am/heev$n.log 2>&1 || { cat gpurun_out/r6/am/heev$n.log; exit 1; }
  echo "n=$n $(grep RESULT gpurun_out/r6/am/heev$n.log)"
done
SLATE_AMD_NATIVE_HEEV_OVERLAP=0 timeout -k 10 300 slate_amd/bench_native heev 16384 256 1 1 1 1 2 0 > gpurun_out/r6/am/serial.log 2>&1 && echo "serial $(grep RESULT gpurun_out/r6/am/serial.log)" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_native_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r6/am/native_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6/am/native_tests.log
exit $rc
