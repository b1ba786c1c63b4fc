#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3f
timeout -k 10 300 python -u -m pytest tests/test_native_gpu.py -x -q -s --timeout 240 --timeout-method thread > gpurun_out/r3f/pytest_native.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/r3f/pytest_native.log
[ $rc -ne 0 ] && exit 1
env -u PYTHONPATH LD_LIBRARY_PATH=/opt/rocm/lib timeout -k 10 200 ./slate_amd/ex_native 1x1 32768 > gpurun_out/r3f/native_32768.log 2>&1; echo "rc=$?"; cat gpurun_out/r3f/native_32768.log
