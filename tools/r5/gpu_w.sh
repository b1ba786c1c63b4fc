#!/bin/bash
# kernel trace of dsyevd n=16384 (last step)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r5/w; mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/heev -o run -- python3 bench.py --routine heev --n 16384 --nb 256 --steps 1 --warmup 1 --check 0 > $D/heev.log 2>&1
echo "prof rc=$?"; tail -1 $D/heev.log | head -c 300
