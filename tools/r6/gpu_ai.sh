#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6/ai
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_native_gpu.py > gpurun_out/r6/ai/native.log 2>&1
rc=$?
grep -E "PASS|FAIL|passed|failed" gpurun_out/r6/ai/native.log | tail -20
exit $rc
