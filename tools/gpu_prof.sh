#!/bin/bash
# Kernel-trace profiles of the headline factorizations on one MI355X, plus
# isolated op timings.  Each GPU step has its own limit; stop at the first failure.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 180 python -u tools/bench_ops.py > gpurun_out/prof/ops.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/potrf -o potrf -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/prof/potrf.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/getrf -o getrf -- python3 bench.py --routine getrf --lookahead 2 --steps 1 --warmup 1 > gpurun_out/prof/getrf.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/geqrf -o geqrf -- python3 bench.py --routine geqrf --m 65536 --n 8192 --nb 256 --steps 1 --warmup 1 > gpurun_out/prof/geqrf.log 2>&1
rc=$?
find gpurun_out/prof -name "*.db" -size +60M -delete
exit $rc
