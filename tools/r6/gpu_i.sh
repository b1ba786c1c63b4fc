#!/bin/bash
# native trace test, then the getrf kernel traces (tools/r6/gpu_h.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6/i; mkdir -p $D
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_native_gpu.py \
  -k "trace or runs_without_python" > $D/native_trace_test.log 2>&1
rc=$?; tail -5 $D/native_trace_test.log; [ $rc -eq 0 ] || exit $rc
bash tools/r6/gpu_h.sh
