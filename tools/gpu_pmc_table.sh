#!/bin/bash
# PMC counters of the hot kernels (one counter pass per workload; each pass
# is its own rocprofv3 run with --pmc only, no trace domains):
#   potrf n=16384 (gemm_real_kernel, potrf_lds_kernel, trsm_rlt_kernel)
#   getrf n=16384 (getrf_base_persist)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
C="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum"
for w in potrf getrf; do
  timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc/$w -o $w -- python3 bench.py --routine $w --n 16384 --steps 1 --warmup 0 --check 0 > gpurun_out/pmc/$w.log 2>&1 || exit 1
done
find gpurun_out/pmc -name "*.csv" -size +50M -delete
exit 0
