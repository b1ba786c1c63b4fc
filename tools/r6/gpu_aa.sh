#!/bin/bash
# native RowMajor getrf: checks + 1-GPU bench (both libraries)
set -o pipefail
mkdir -p gpurun_out/r6/aa
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_native_gpu.py -k "example" > gpurun_out/r6/aa/native.log 2>&1
rc=$?
tail -3 gpurun_out/r6/aa/native.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --impl native --routine getrf --steps 5 --warmup 2 > gpurun_out/r6/aa/getrf_native.json 2> gpurun_out/r6/aa/getrf_native.err
rc=$?
tail -1 gpurun_out/r6/aa/getrf_native.json
[ $rc -ne 0 ] && { tail -5 gpurun_out/r6/aa/getrf_native.err; exit $rc; }
SLATE_AMD_NATIVE_LU_ROWMAJOR=0 timeout -k 10 300 python -u bench.py --impl native --routine getrf --steps 5 --warmup 2 > gpurun_out/r6/aa/getrf_native_cm.json 2>/dev/null
tail -1 gpurun_out/r6/aa/getrf_native_cm.json
