#!/bin/bash
# clock + MFMA-busy counters of the dgemm bench (one counter pass)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/pmc/gemm -o gemm --output-format csv -- python3 bench.py --routine gemm --n 16384 --steps 1 --warmup 0 --check 0 > gpurun_out/pmc/gemm.log 2>&1
