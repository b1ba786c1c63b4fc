#!/bin/bash
# Python dgetrf kernel trace (compare with the native RowMajor path)
set -o pipefail
mkdir -p gpurun_out/r6/ac
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r6/ac/prof_py -o py -- python3 $GRAFT_REPO_ROOT/bench.py --routine getrf --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r6/ac/py.log 2>&1
echo "py rc=$?"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r6/ac/prof_nat -o nat -- $GRAFT_REPO_ROOT/slate_amd/bench_native getrf 32768 512 1 1 1 1 2 0 > $GRAFT_REPO_ROOT/gpurun_out/r6/ac/nat.log 2>&1
echo "nat rc=$?"
