#!/bin/bash
# dpotrf kernel profile (GEMM coverage per tenth of the factorization)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${TAG:-s11}; mkdir -p $D
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof_potrf -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --check 0 > $GRAFT_REPO_ROOT/$D/prof_potrf.log 2>&1
echo "prof rc=$?"; grep metric $GRAFT_REPO_ROOT/$D/prof_potrf.log | cut -c1-150
