#!/bin/bash
# getrf: dynamic panel-CU reservation (levels of 8 CUs) vs fixed 64
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sweep_w
timeout -k 10 300 python -u -m pytest tests/test_dist_gpu.py -m gpu -x -q -k "getrf" --timeout 200 --timeout-method thread > gpurun_out/sweep_w/pytest.log 2>&1 || { tail -30 gpurun_out/sweep_w/pytest.log; exit 1; }
tail -1 gpurun_out/sweep_w/pytest.log
for dyn in 1 0; do
  SLATE_AMD_LU_DYNCU=$dyn timeout -k 10 150 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 > gpurun_out/sweep_w/getrf_dyn$dyn.log 2>&1 || exit 1
  echo "dyn=$dyn $(grep -o '"value": [0-9.]*\|"residual": [0-9.e-]*' gpurun_out/sweep_w/getrf_dyn$dyn.log | tr '\n' ' ')"
done
SLATE_AMD_LU_DYNCU=1 timeout -k 10 150 python -u bench.py --routine getrf --lookahead 1 --steps 3 --warmup 1 --check 0 > gpurun_out/sweep_w/getrf_la1.log 2>&1 || exit 1
echo "dyn=1 la=1 $(grep -o '"value": [0-9.]*' gpurun_out/sweep_w/getrf_la1.log)"
