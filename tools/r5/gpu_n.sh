#!/bin/bash
# benches after routing the small fp64 GEMMs to glds, then one kernel trace (last: the profiler can crash at teardown)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r5/n; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_native_gpu.py -x -q --timeout 240 --timeout-method thread > $D/tests.log 2>&1
rc=$?; tail -2 $D/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $D/tests.log | head; exit 1; }
timeout -k 10 200 python -u bench.py > $D/bench_potrf.log 2>&1 || { tail $D/bench_potrf.log; exit 1; }
tail -1 $D/bench_potrf.log
timeout -k 10 200 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 > $D/bench_getrf.log 2>&1 || { tail $D/bench_getrf.log; exit 1; }
tail -1 $D/bench_getrf.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/potrf -o run -- python3 bench.py --steps 2 --warmup 1 --check 0 > $D/potrf_prof.log 2>&1
echo "prof rc=$?"
