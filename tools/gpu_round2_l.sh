#!/bin/bash
# stedc GPU merge test, heev phases, kernel stats of heev
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_eig_svd.py -x -v --timeout 150 --timeout-method thread -m gpu > gpurun_out/pytest_eig.log 2>&1 || { tail -40 gpurun_out/pytest_eig.log; exit 1; }
tail -3 gpurun_out/pytest_eig.log
SLATE_AMD_HB2ST=device timeout -k 10 300 python -u tools/heev_phases.py 16384 256 > gpurun_out/heev_phases.log 2>&1 || { cat gpurun_out/heev_phases.log; exit 1; }
cat gpurun_out/heev_phases.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_heev -o heev -- python3 tools/heev_phases.py 8192 256 > gpurun_out/prof_heev.log 2>&1 || { tail gpurun_out/prof_heev.log; exit 1; }
find gpurun_out/prof_heev -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -25 {}'
