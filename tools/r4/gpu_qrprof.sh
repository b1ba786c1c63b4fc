#!/bin/bash
# kernel stats of the native and the Python dgeqrf (m=65536, n=8192)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4/qrprof
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4/qrprof/native -o run -- $R/slate_amd/bench_native geqrf 8192 512 1 1 1 0 1 0 65536 > $R/gpurun_out/r4/qrprof/native.log 2>&1 &&
cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4/qrprof/py -o run -- python bench.py --routine geqrf --m 65536 --n 8192 --steps 1 --warmup 1 > $R/gpurun_out/r4/qrprof/py.log 2>&1
rc=$?
find $R/gpurun_out/r4/qrprof -name "*stats*" | head
exit $rc
