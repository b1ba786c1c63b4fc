#!/bin/bash
# native distributed heev + redistribute (ex_native 1x1 and host-transport grids), census
set -o pipefail
mkdir -p gpurun_out/r6/t
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_native_gpu.py -k "example" > gpurun_out/r6/t/native.log 2>&1
rc=$?
tail -15 gpurun_out/r6/t/native.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_kernel_census_gpu.py > gpurun_out/r6/t/census.log 2>&1
rc=$?
tail -8 gpurun_out/r6/t/census.log
exit $rc
