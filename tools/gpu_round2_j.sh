#!/bin/bash
# Re-entry check after the container was restored: gpu tests, smoke,
# headline benches, heev (host vs device bulge chase), potrf kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_check.sh &&
timeout -k 10 300 python -u bench.py --routine heev --n 16384 --nb 256 --steps 1 --warmup 1 > gpurun_out/bench_heev.log 2>&1 &&
SLATE_AMD_HB2ST=device timeout -k 10 300 python -u bench.py --routine heev --n 16384 --nb 256 --steps 1 --warmup 1 > gpurun_out/bench_heev_dev.log 2>&1
echo "exit $?"
grep -h '"metric"' gpurun_out/bench_*.log
tail -3 gpurun_out/pytest_gpu.log
