#!/bin/bash
# he2hb fused rank-2k update + explicit V^H in the back-transforms: tests, dsyevd phases and bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
SLATE_AMD_QR_VH_ROWS=1 timeout -k 10 400 python -u -m pytest tests/test_eig_svd.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_aj.log 2>&1 || { tail -30 gpurun_out/pytest_aj.log; exit 1; }
tail -1 gpurun_out/pytest_aj.log
timeout -k 10 300 python -u tools/heev_phases.py 16384 256 > gpurun_out/heev_phases.log 2>&1 || { tail gpurun_out/heev_phases.log; exit 1; }
tail -12 gpurun_out/heev_phases.log
timeout -k 10 300 python -u bench.py --routine heev --n 16384 --nb 256 --steps 1 --warmup 1 > gpurun_out/bench_heev.log 2>&1 || { tail gpurun_out/bench_heev.log; exit 1; }
grep -h '"metric"' gpurun_out/bench_heev.log
