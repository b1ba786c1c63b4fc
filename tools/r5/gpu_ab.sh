#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r5/ab; mkdir -p $D
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_IFETCH SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --kernel-trace --output-format csv -d $D/p2 -o run -- python3 tools/r5/lu_panel_one.py 8192 > $D/p2.log 2>&1
echo "pmc2 rc=$?"
