#!/bin/bash
# native matrix model checks (1x1 and the host-transport grids), then the getrf sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6/k; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_native_gpu.py \
  -k "runs_without_python or grids_host_transport" > $D/native_tests.log 2>&1
rc=$?; tail -6 $D/native_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/r6/gpu_j.sh
