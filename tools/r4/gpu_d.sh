#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/r4/scal_repro.py 2 || exit 1
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_native_gpu.py > gpurun_out/native3.log 2>&1; echo "native rc=$?"; tail -2 gpurun_out/native3.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_nosync_gpu.py tests/test_kernels_gpu.py tests/test_lu_rowmajor_gpu.py > gpurun_out/gpu_d.log 2>&1; echo "gpu rc=$?"; tail -3 gpurun_out/gpu_d.log
