#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6/v
timeout -k 10 600 python -u tools/r6/heev_grid_sweep.py > gpurun_out/r6/v/sweep.log 2>&1
rc=$?
cat gpurun_out/r6/v/sweep.log | tail -30
exit $rc
