#!/bin/bash
# native LAPACK / ScaLAPACK additions from C, then the 1-GPU potrf trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r6; mkdir -p $D
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_native_gpu.py \
  -k "lapack_more or scalapack_from_c or exports" > $D/pytest_c.log 2>&1
rc=$?; tail -15 $D/pytest_c.log; [ $rc -eq 0 ] || exit $rc
./tools/r6/gpu_b.sh
