#!/bin/bash
# Session re-entry check: full GPU test suite, smoke, default bench (dpotrf), dgetrf bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s1/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/s1/pytest_gpu.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 200 python -u bench.py > gpurun_out/s1/bench_potrf.log 2>&1 || { tail gpurun_out/s1/bench_potrf.log; exit 1; }
tail -1 gpurun_out/s1/bench_potrf.log
timeout -k 10 200 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 > gpurun_out/s1/bench_getrf.log 2>&1 || { tail gpurun_out/s1/bench_getrf.log; exit 1; }
tail -1 gpurun_out/s1/bench_getrf.log
timeout -k 10 200 python -u tools/probe/lu_panel_time.py > gpurun_out/s1/lu_panel_time.log 2>&1 || { tail gpurun_out/s1/lu_panel_time.log; exit 1; }
cat gpurun_out/s1/lu_panel_time.log
