#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_eig_svd.py -x -q --timeout 150 --timeout-method thread -m gpu > gpurun_out/pytest_eig.log 2>&1 || { tail -30 gpurun_out/pytest_eig.log; exit 1; }
tail -1 gpurun_out/pytest_eig.log
for th in 256 512 1024; do
  SLATE_AMD_HB2ST=device SLATE_AMD_HB2ST_THREADS=$th timeout -k 10 200 python -u tools/heev_phases.py 16384 256 > gpurun_out/heev_th$th.log 2>&1 || { cat gpurun_out/heev_th$th.log; exit 1; }
  echo "threads=$th"; grep -E "heev n=|device   hb2st" gpurun_out/heev_th$th.log
done
