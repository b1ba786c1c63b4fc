#!/bin/bash
# one kernel-trace profile (the rocprof step is last: its teardown may segfault)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
name=$1; shift
mkdir -p gpurun_out/prof_$name
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$name -o $name -- python3 "$@" > gpurun_out/prof_$name/run.log 2>&1
rc=$?
find gpurun_out/prof_$name -name "*.db" -size +60M -delete
exit $rc
