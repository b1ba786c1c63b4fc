#!/bin/bash
# getrf persistent panel: rows per thread (1/2/4) x reserved panel CUs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sweep_y
SLATE_AMD_LU_RPT=4 timeout -k 10 300 python -u -m pytest tests/test_dist_gpu.py tests/test_kernels_gpu.py -m gpu -x -q -k "getrf or lu" --timeout 200 --timeout-method thread > gpurun_out/sweep_y/pytest.log 2>&1 || { tail -30 gpurun_out/sweep_y/pytest.log; exit 1; }
tail -1 gpurun_out/sweep_y/pytest.log
for cfg in "1 64" "2 32" "2 40" "4 16" "4 24"; do
  set -- $cfg
  SLATE_AMD_LU_RPT=$1 SLATE_AMD_PANEL_CUS=$2 timeout -k 10 150 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 > gpurun_out/sweep_y/getrf_r$1_c$2.log 2>&1 || exit 1
  echo "rpt=$1 cus=$2 $(grep -o '"value": [0-9.]*\|"residual": [0-9.e-]*' gpurun_out/sweep_y/getrf_r$1_c$2.log | tr '\n' ' ')"
done
