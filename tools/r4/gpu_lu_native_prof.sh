#!/bin/bash
# kernel totals of the native and the Python dgetrf (n = 32768): summaries only
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/lunat -o run -- $R/slate_amd/bench_native getrf 32768 512 1 1 1 1 1 0 32768 > $R/gpurun_out/r4/lu_native_prof.log 2>&1 &&
cd $R && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/lupy -o run -- python3 bench.py --routine getrf --steps 1 --warmup 1 > $R/gpurun_out/r4/lu_py_prof.log 2>&1
rc=$?
for d in lunat lupy; do
  f=$(find /tmp/$d -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && head -25 "$f" > $R/gpurun_out/r4/${d}_kernel_stats.csv
done
exit $rc
