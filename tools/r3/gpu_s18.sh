#!/bin/bash
# LU publishers arrive directly; tb2bd store drain: full GPU suite, LU panel latency, dgetrf bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${TAG:-s18}; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $D/pytest.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 200 python -u tools/probe/lu_panel_time.py > $D/lu_panel_time.log 2>&1 || { tail $D/lu_panel_time.log; exit 1; }
grep "m=  8192\|m= 32768" $D/lu_panel_time.log
timeout -k 10 200 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 > $D/bench_getrf.log 2>&1 || { tail $D/bench_getrf.log; exit 1; }
tail -1 $D/bench_getrf.log | cut -c1-200
