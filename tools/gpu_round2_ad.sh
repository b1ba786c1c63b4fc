#!/bin/bash
# tb2bd: 1024 threads, lag 4 -- correctness + timing; chase with 128 KB staging
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_eig_svd.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ad.log 2>&1 || { tail -30 gpurun_out/pytest_ad.log; exit 1; }
tail -1 gpurun_out/pytest_ad.log
timeout -k 10 300 python -u tools/probe/tb2bd_time.py 8192 64
SLATE_AMD_TB2BD_LAG=8 timeout -k 10 300 python -u tools/probe/tb2bd_time.py 8192 64 | head -1
timeout -k 10 300 python -u bench.py --routine heev --n 16384 --nb 256 --steps 1 --warmup 1 > gpurun_out/bench_heev.log 2>&1 || { tail gpurun_out/bench_heev.log; exit 1; }
grep -h '"metric"' gpurun_out/bench_heev.log
