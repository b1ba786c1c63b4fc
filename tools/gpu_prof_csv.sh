#!/bin/bash
# one rocprofv3 kernel-trace run with CSV output (the rocprof step is the
# last GPU step of a call: its teardown may segfault after writing output)
#   bash tools/gpu_prof_csv.sh <name> <bench.py args...>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
name=$1; shift
mkdir -p gpurun_out/pc_$name
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pc_$name -o $name -- python3 bench.py "$@" > gpurun_out/pc_$name/run.log 2>&1
rc=$?
find gpurun_out/pc_$name -name "*kernel_trace.csv" -size +50M -delete
exit $rc
