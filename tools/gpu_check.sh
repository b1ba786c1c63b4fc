#!/bin/bash
# One GPU-box pass: gpu tests, smoke, headline benches.  Each GPU step has its
# own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 180 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench_potrf.log 2>&1 &&
timeout -k 10 180 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 > gpurun_out/bench_getrf.log 2>&1 &&
timeout -k 10 180 python -u bench.py --routine gemm --n 16384 --steps 3 --warmup 1 > gpurun_out/bench_gemm.log 2>&1 &&
timeout -k 10 180 python -u bench.py --routine geqrf --m 65536 --n 8192 --nb 256 --steps 2 --warmup 1 > gpurun_out/bench_geqrf.log 2>&1
