#!/bin/bash
# native library: tests (grids on one GPU through the host transport) and the
# bench.py --impl native headline runs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v -s --timeout 400 --timeout-method thread tests/test_native_gpu.py > gpurun_out/native2.log 2>&1 || { echo "native tests rc=$?"; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/native2.log
for r in potrf getrf gemm; do
  timeout -k 10 300 python -u bench.py --impl native --routine $r --steps 3 --warmup 1 > gpurun_out/bench_native_$r.log 2>&1 || { echo "bench $r rc=$?"; cat gpurun_out/bench_native_$r.log; exit 1; }
  tail -1 gpurun_out/bench_native_$r.log
done
