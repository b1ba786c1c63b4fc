#!/bin/bash
# kernel trace of the op micro-benchmarks (single rocprof run; last step)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tops
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/tops -o ops --output-format csv -- python3 tools/bench_ops.py > gpurun_out/tops/ops.log 2>&1
