#!/bin/bash
# native heev: 1-GPU n=16384 stage trace + ex_native checks (1x1, grids)
set -o pipefail
bash tools/r6/gpu_x.sh || exit $?
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_native_gpu.py -k "example" > gpurun_out/r6/x/native.log 2>&1
rc=$?
tail -5 gpurun_out/r6/x/native.log
exit $rc
