#!/bin/bash
# PMC counters of the heev kernels (n = 8192), one --pmc pass
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/pmc_r3h; mkdir -p $D
C="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum"
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $D/heev -o heev -- python3 bench.py --routine heev --n 8192 --nb 256 --steps 1 --warmup 0 --check 0 > $D/heev.log 2>&1
rc=$?; echo "rc=$rc"; tail -5 $D/heev.log
find $D -name "*.csv" -size +50M -delete
exit $rc
