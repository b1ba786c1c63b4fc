#!/bin/bash
# kernel trace of the 1-GPU dpotrf / dgetrf benches after the glds GEMM
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r5/l; mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/potrf -o run -- python3 bench.py --steps 2 --warmup 1 --check 0 > $D/potrf.log 2>&1 || { tail $D/potrf.log; exit 1; }
tail -1 $D/potrf.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/getrf -o run -- python3 bench.py --routine getrf --lookahead 2 --steps 2 --warmup 1 --check 0 > $D/getrf.log 2>&1 || { tail $D/getrf.log; exit 1; }
tail -1 $D/getrf.log
find $D -name "*stats*" | head
