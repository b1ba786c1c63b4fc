#!/bin/bash
# round 6: kernel census incl. hetrf + 2-rank heev/hetrf, stedc merge, hesv, condest
set -o pipefail
mkdir -p gpurun_out/r6/r
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_kernel_census_gpu.py tests/test_eig_svd.py -k "stedc or hesv or hetrf or census or own_kernels" \
  tests/test_band_indef.py -m gpu > gpurun_out/r6/r/census.log 2>&1
rc=$?
tail -25 gpurun_out/r6/r/census.log
exit $rc
