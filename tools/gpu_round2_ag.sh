#!/bin/bash
# geqrf: 64x64 small-tile threshold sweep (the split-K V^T C GEMMs)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sweep_ag
for th in 2048 1024 512 0; do
  SLATE_AMD_GEMM_SMALL=$th timeout -k 10 150 python -u bench.py --routine geqrf --m 65536 --n 8192 --nb 256 --steps 3 --warmup 1 --check 0 > gpurun_out/sweep_ag/geqrf_s$th.log 2>&1 || exit 1
  echo "small=$th $(grep -o '"value": [0-9.]*' gpurun_out/sweep_ag/geqrf_s$th.log)"
done
timeout -k 10 150 python -u tools/exp/gemm_tn.py > gpurun_out/sweep_ag/gemm_tn.log 2>&1 && tail -8 gpurun_out/sweep_ag/gemm_tn.log
SLATE_AMD_GEMM_SMALL=0 timeout -k 10 150 python -u tools/exp/gemm_tn.py > gpurun_out/sweep_ag/gemm_tn0.log 2>&1 && tail -8 gpurun_out/sweep_ag/gemm_tn0.log
