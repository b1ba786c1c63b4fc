#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4/heevprof
cd $R && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r4/heevprof -o run -- python bench.py --routine heev --n 16384 --steps 1 --warmup 1 > $R/gpurun_out/r4/heevprof/log.txt 2>&1
