#!/bin/bash
# quad-lane compute in the fused chase task: eig GPU tests + chase timing + dsyevd bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_eig_svd.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_an.log 2>&1 || { tail -30 gpurun_out/pytest_an.log; exit 1; }
tail -1 gpurun_out/pytest_an.log
timeout -k 10 200 python -u tools/probe/hb2st_time.py 16384 64 > gpurun_out/hb2st_quad.log 2>&1 || { tail gpurun_out/hb2st_quad.log; exit 1; }
grep -h 'device\|phases\|eig diff' gpurun_out/hb2st_quad.log
timeout -k 10 300 python -u bench.py --routine heev --n 16384 --nb 256 --steps 1 --warmup 1 > gpurun_out/bench_heev.log 2>&1 || { tail gpurun_out/bench_heev.log; exit 1; }
grep -h '"metric"' gpurun_out/bench_heev.log | cut -c1-200
