#!/bin/bash
# heev with Q1 formed during the chase: GPU eig tests, OOC tests, bench both ways
set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_eig_svd.py -m gpu > gpurun_out/r4/heevq1_tests.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_nosync_gpu.py -k out_of_core > gpurun_out/r4/ooc_tests.log 2>&1 &&
timeout -k 10 240 python bench.py --routine heev --n 16384 --steps 2 --warmup 1 > gpurun_out/r4/bench_heev_q1.log 2>&1 &&
SLATE_AMD_HEEV_Q1=0 timeout -k 10 240 python bench.py --routine heev --n 16384 --steps 2 --warmup 1 > gpurun_out/r4/bench_heev_noq1.log 2>&1
rc=$?
tail -2 gpurun_out/r4/heevq1_tests.log gpurun_out/r4/ooc_tests.log
grep -h metric gpurun_out/r4/bench_heev_q1.log gpurun_out/r4/bench_heev_noq1.log | cut -c1-200
exit $rc
