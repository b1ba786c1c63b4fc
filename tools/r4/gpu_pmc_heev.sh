#!/bin/bash
# PMC pass over dsyevd n = 8192: LDS conflicts / MFMA busy of the stage-2 kernels
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4
cd $R && timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d /tmp/pmc_heev -o run -- python3 bench.py --routine heev --n 8192 --steps 1 --warmup 0 > $R/gpurun_out/r4/pmc_heev_log.txt 2>&1
rc=$?
python3 tools/prof/pmc_csv_summary.py /tmp/pmc_heev > $R/gpurun_out/r4/pmc_heev_n8192_r4.txt 2>&1
exit $rc
