#!/bin/bash
# instruction-fetch counters of the LU panel base kernel (the fully unrolled 32-column loop)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r5/aa; mkdir -p $D
timeout -s KILL 60 rocprofv3 -L > $D/avail.txt 2>&1; grep -oE "SQ[C]?_[A-Z_]*(ICACHE|INST|IFETCH)[A-Z_]*" $D/avail.txt | sort -u | head -40
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $D/p1 -o run -- python3 tools/r5/lu_panel_one.py 8192 > $D/p1.log 2>&1
echo "pmc1 rc=$?"
