#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --routine heev --n 16384 --nb 256 --steps 2 --warmup 1 > gpurun_out/b_heev.log 2>&1; echo "heev rc=$?"; tail -1 gpurun_out/b_heev.log | cut -c1-300
timeout -k 10 400 python -u bench.py --routine geqrf --m 65536 --n 8192 --nb 256 --steps 3 --warmup 1 > gpurun_out/b_geqrf.log 2>&1; echo "geqrf rc=$?"; tail -1 gpurun_out/b_geqrf.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_heev -o heev -- python3 bench.py --routine heev --n 16384 --nb 256 --steps 1 --warmup 1 --check 0 > gpurun_out/prof_heev.log 2>&1; echo "prof rc=$?"
find gpurun_out/prof_heev -name "*kernel_stats.csv" | head -2
