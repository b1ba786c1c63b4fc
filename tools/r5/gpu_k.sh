#!/bin/bash
# glds GEMM: second variant sweep, the GEMM/BLAS-3 GPU tests on the new
# default, then the potrf / getrf / dgemm benches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/k; mkdir -p $D
timeout -k 10 200 ./tools/exp/dgemm_glds_r5.bin > $D/sweep2.txt 2>&1 || { tail -5 $D/sweep2.txt; exit 1; }
grep -c "rel 0.000e+00" $D/sweep2.txt
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_native_gpu.py -x -q --timeout 240 --timeout-method thread > $D/tests.log 2>&1
rc=$?; tail -3 $D/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $D/tests.log | head; exit 1; }
timeout -k 10 200 python -u bench.py > $D/bench_potrf.log 2>&1 || { tail $D/bench_potrf.log; exit 1; }
tail -1 $D/bench_potrf.log
timeout -k 10 200 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 > $D/bench_getrf.log 2>&1 || { tail $D/bench_getrf.log; exit 1; }
tail -1 $D/bench_getrf.log
timeout -k 10 200 python -u bench.py --routine gemm --steps 3 --warmup 1 > $D/bench_gemm.log 2>&1 || { tail $D/bench_gemm.log; exit 1; }
tail -1 $D/bench_gemm.log
