#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6/u
timeout -k 10 600 python -u tools/r6/heev_grid_bench.py 1gpu grid > gpurun_out/r6/u/heev.log 2>&1
rc=$?
cat gpurun_out/r6/u/heev.log | tail -30
[ $rc -ne 0 ] && exit $rc
PYTHONPATH=$PWD:$PWD/tests timeout -k 10 300 python -u tools/r6/census_stack.py > gpurun_out/r6/s/stack.log 2>&1
grep -A12 "^SPY" gpurun_out/r6/s/stack.log | head -40
grep "^\[he" gpurun_out/r6/s/stack.log
