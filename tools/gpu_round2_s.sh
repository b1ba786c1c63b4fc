#!/bin/bash
# Re-validation after a fresh rebuild: GPU tests, smoke, all headline benches.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 180 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench_potrf.log 2>&1 || { tail gpurun_out/bench_potrf.log; exit 1; }
timeout -k 10 180 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 > gpurun_out/bench_getrf.log 2>&1 || { tail gpurun_out/bench_getrf.log; exit 1; }
timeout -k 10 180 python -u bench.py --routine gemm --n 16384 --steps 3 --warmup 1 > gpurun_out/bench_gemm.log 2>&1 || { tail gpurun_out/bench_gemm.log; exit 1; }
timeout -k 10 180 python -u bench.py --routine geqrf --m 65536 --n 8192 --nb 256 --steps 2 --warmup 1 > gpurun_out/bench_geqrf.log 2>&1 || { tail gpurun_out/bench_geqrf.log; exit 1; }
timeout -k 10 300 python -u bench.py --routine heev --n 16384 --nb 256 --steps 1 --warmup 1 > gpurun_out/bench_heev.log 2>&1 || { tail gpurun_out/bench_heev.log; exit 1; }
grep -h '"metric"' gpurun_out/bench_*.log
