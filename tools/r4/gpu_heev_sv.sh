#!/bin/bash
# reflector LDS pitch change: hb2st / heev GPU tests, then the dsyevd bench
set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_eig_svd.py -m gpu > gpurun_out/r4/heev_sv_tests.log 2>&1 &&
timeout -k 10 240 python bench.py --routine heev --n 16384 --steps 2 --warmup 1 > gpurun_out/r4/bench_heev_sv.log 2>&1
rc=$?
tail -n 2 gpurun_out/r4/heev_sv_tests.log
grep -h metric gpurun_out/r4/bench_heev_sv.log | cut -c1-160
exit $rc
