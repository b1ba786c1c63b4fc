#!/bin/bash
# quick GPU iteration: selected kernel tests, op timings, headline bench
set -o pipefail
mkdir -p gpurun_out
K=${K:-"fast or potrf or trsm"}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/quick_tests.log 2>&1 &&
timeout -k 10 120 python -u tools/bench_ops.py > gpurun_out/quick_ops.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 > gpurun_out/quick_bench.log 2>&1
