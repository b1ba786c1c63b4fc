#!/bin/bash
# round-end rehearsal on the current tree: full GPU suite, smoke, default bench (dpotrf), dgetrf / dgeqrf / dsyevd / dgemm benches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${TAG:-r4base}; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $D/pytest.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 200 python -u bench.py > $D/bench_potrf.log 2>&1 || { tail $D/bench_potrf.log; exit 1; }
tail -1 $D/bench_potrf.log
timeout -k 10 200 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 > $D/bench_getrf.log 2>&1 || { tail $D/bench_getrf.log; exit 1; }
tail -1 $D/bench_getrf.log
timeout -k 10 200 python -u bench.py --routine geqrf --rows 65536 --size 8192 --nb 256 --steps 3 --warmup 1 > $D/bench_geqrf.log 2>&1 || { tail $D/bench_geqrf.log; exit 1; }
tail -1 $D/bench_geqrf.log
timeout -k 10 300 python -u bench.py --routine heev --n 16384 --nb 256 --steps 2 --warmup 1 > $D/bench_heev.log 2>&1 || { tail $D/bench_heev.log; exit 1; }
tail -1 $D/bench_heev.log
timeout -k 10 300 python -u bench.py --routine gemm --steps 3 --warmup 1 > $D/bench_gemm.log 2>&1 || { tail $D/bench_gemm.log; exit 1; }
tail -1 $D/bench_gemm.log
timeout -k 10 200 python -u tools/probe/lu_panel_time.py > $D/lu_panel.log 2>&1 || { tail $D/lu_panel.log; exit 1; }
tail -3 $D/lu_panel.log
