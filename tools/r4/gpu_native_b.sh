#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for n in 2048 8192 32768; do
  for r in potrf getrf gemm; do
    timeout -k 10 200 ./slate_amd/bench_native $r $n 512 1 1 1 1 2 1 > gpurun_out/bn_${r}_$n.log 2>&1 || { echo "rc=$? $r $n"; cat gpurun_out/bn_${r}_$n.log; exit 1; }
    echo "$r $n: $(tr '\n' ' ' < gpurun_out/bn_${r}_$n.log)"
  done
done
