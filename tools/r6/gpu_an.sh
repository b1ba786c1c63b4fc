#!/bin/bash
# native heev: he2hb lookahead (panel QR on the side stream) on / off
set -o pipefail
mkdir -p gpurun_out/r6/an
for n in 4096 16384; do
  timeout -k 10 300 slate_amd/bench_native heev $n 256 1 1 1 1 3 1 > gpurun_out/r6/an/heev$n.log 2>&1 || { cat gpurun_out/r6/an/heev$n.log; exit 1; }
  echo "n=$n $(grep RESULT gpurun_out/r6/an/heev$n.log)"
done
SLATE_AMD_NATIVE_HE2HB_LOOKAHEAD=0 timeout -k 10 300 slate_amd/bench_native heev 16384 256 1 1 1 1 3 0 > gpurun_out/r6/an/nola.log 2>&1 && echo "no lookahead $(grep RESULT gpurun_out/r6/an/nola.log)" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_native_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r6/an/native_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6/an/native_tests.log
exit $rc
