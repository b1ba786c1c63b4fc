#!/bin/bash
# rocprofv3 kernel stats of the native dsyevd n=16384 (1 warm-up + 1 step)
set -o pipefail
mkdir -p gpurun_out/r6/aq
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r6/aq/prof -o heev -- $GRAFT_REPO_ROOT/slate_amd/bench_native heev 16384 256 1 1 1 1 1 0 > $GRAFT_REPO_ROOT/gpurun_out/r6/aq/prof.log 2>&1
rc=$?
grep RESULT $GRAFT_REPO_ROOT/gpurun_out/r6/aq/prof.log
echo "rocprof rc=$rc"
exit $rc
