#!/bin/bash
# geqrf: explicit V^H (NN trailing V^H C) vs TN
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sweep_ah
timeout -k 10 300 python -u -m pytest tests/test_qr.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sweep_ah/pytest.log 2>&1 || { tail -30 gpurun_out/sweep_ah/pytest.log; exit 1; }
tail -1 gpurun_out/sweep_ah/pytest.log
for r in 4096 0 4096 0; do
  SLATE_AMD_QR_VH_ROWS=$r timeout -k 10 150 python -u bench.py --routine geqrf --m 65536 --n 8192 --nb 256 --steps 3 --warmup 1 > gpurun_out/sweep_ah/geqrf_v$r.log 2>&1 || exit 1
  echo "vh_rows=$r $(grep -o '"value": [0-9.]*\|"residual": [0-9.e-]*' gpurun_out/sweep_ah/geqrf_v$r.log | tr '\n' ' ')"
done
