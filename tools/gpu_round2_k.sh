#!/bin/bash
# devpool tests, potrf sweep (diag block, group), heev phase breakdown,
# potrf kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python -u -m pytest tests/test_devpool_gpu.py -x -v --timeout 60 --timeout-method thread > gpurun_out/pytest_devpool.log 2>&1 || { tail -30 gpurun_out/pytest_devpool.log; exit 1; }
tail -3 gpurun_out/pytest_devpool.log
for cfg in "256 2" "512 2" "256 1" "256 3"; do
  set -- $cfg
  v=$(SLATE_AMD_POTRF_DIAG=$1 SLATE_AMD_POTRF_GROUP=$2 timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 2>&1 | grep -o '"value": [0-9.]*' | tr '\n' ' ') || exit 1
  echo "diag=$1 group=$2 $v"
done
SLATE_AMD_HB2ST=device timeout -k 10 300 python -u tools/heev_phases.py 16384 256 > gpurun_out/heev_phases.log 2>&1 || exit 1
cat gpurun_out/heev_phases.log
