#!/bin/bash
# native C ABI checks (C++ header API over the native library, LAPACK
# extras, handles), then the per-link 2x4 projections (tools/r6/gpu_p.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6/q; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_native_gpu.py \
  -k "cpp_header or lapack_more or handle_capi" > $D/native_tests.log 2>&1
rc=$?; tail -8 $D/native_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/r6/gpu_p.sh
