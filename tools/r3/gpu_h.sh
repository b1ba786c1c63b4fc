#!/bin/bash
# hipGraph capture probe, stream census test, GPU stedc tests + timing,
# heev bench, getrf (laswp pitch + deferred left swaps) and potrf benches.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3h
mkdir -p $O
timeout -k 10 240 python -u -m pytest tests/test_eig_svd.py tests/test_nosync_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_eig_nosync.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 $O/pytest_eig_nosync.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 120 python -u tools/probe/stedc_time.py 4096 > $O/stedc_4096.log 2>&1 || { echo stedc4096 failed; tail $O/stedc_4096.log; exit 1; }
cat $O/stedc_4096.log
timeout -k 10 180 python -u tools/probe/stedc_time.py 16384 > $O/stedc_16384.log 2>&1 || { echo stedc16384 failed; tail $O/stedc_16384.log; exit 1; }
cat $O/stedc_16384.log
timeout -k 10 240 python -u bench.py --routine heev --n 16384 --nb 256 --steps 1 --warmup 1 > $O/bench_heev.log 2>&1 || { echo heev bench failed; tail $O/bench_heev.log; exit 1; }
tail -1 $O/bench_heev.log
timeout -k 10 200 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 > $O/bench_getrf.log 2>&1 || { echo getrf bench failed; tail $O/bench_getrf.log; exit 1; }
tail -1 $O/bench_getrf.log
SLATE_AMD_LU_LEFT_TAIL=0 timeout -k 10 200 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 > $O/bench_getrf_tail0.log 2>&1 || { echo getrf bench failed; exit 1; }
tail -1 $O/bench_getrf_tail0.log
timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 > $O/bench_potrf.log 2>&1 || { echo potrf bench failed; tail $O/bench_potrf.log; exit 1; }
tail -1 $O/bench_potrf.log
timeout -k 10 180 python -u tools/probe/graph_probe.py > $O/graph_probe.log 2>&1
rc=$?; echo "graph probe rc=$rc"; tail -20 $O/graph_probe.log
exit $rc
