#!/bin/bash
# full GPU suite + smoke + getrf default (2 rows/thread, 32 reserved CUs) + getrf kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 180 python -u bench.py --routine getrf --lookahead 2 --steps 5 --warmup 2 > gpurun_out/bench_getrf.log 2>&1 || { tail gpurun_out/bench_getrf.log; exit 1; }
grep -h '"metric"' gpurun_out/bench_getrf.log
bash tools/gpu_prof_csv.sh getrf --routine getrf --lookahead 2 --steps 1 --warmup 1
