#!/bin/bash
# full GPU suite + headline benches (python and native)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/gpu_all.log 2>&1; echo "gpu-all rc=$?"; tail -4 gpurun_out/gpu_all.log
for r in potrf getrf gemm; do
  timeout -k 10 300 python -u bench.py --impl native --routine $r --steps 3 --warmup 1 > gpurun_out/bn_$r.log 2>&1; echo "native $r rc=$?"; tail -1 gpurun_out/bn_$r.log | cut -c1-330
done
