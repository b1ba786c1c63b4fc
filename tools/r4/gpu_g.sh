#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_potrf -o potrf -- python3 bench.py --routine potrf --steps 1 --warmup 1 --check 0 > gpurun_out/prof_potrf.log 2>&1; echo "prof potrf rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_getrf -o getrf -- python3 bench.py --routine getrf --lookahead 2 --steps 1 --warmup 1 --check 0 > gpurun_out/prof_getrf.log 2>&1; echo "prof getrf rc=$?"
ls gpurun_out/prof_potrf gpurun_out/prof_getrf
