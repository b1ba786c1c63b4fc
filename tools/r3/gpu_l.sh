#!/bin/bash
# PMC pass over heev n=8192 (hb2st_kernel, unmtr_hb2st_mfma_kernel, stedc kernels)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && export PYTHONPATH="$GRAFT_REPO_ROOT"
O=gpurun_out/r3l
mkdir -p $O
C="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum"
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $O/pmc_heev -o heev -- python3 bench.py --routine heev --n 8192 --nb 256 --steps 1 --warmup 0 --check 0 > $O/pmc_heev.log 2>&1
rc=$?; echo "pmc rc=$rc"
python3 tools/pmc_summary.py $O/pmc_heev 14 > $O/pmc_heev.txt 2>&1; grep -v raw $O/pmc_heev.txt | head -20
find $O -name "*.csv" -size +40M -delete
exit 0
