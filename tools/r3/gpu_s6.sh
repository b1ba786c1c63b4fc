#!/bin/bash
# heev after column preload + parallelogram k-steps; dgetrf kernel profile with GEMM coverage per tenth
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${TAG:-s6}; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_eig_svd.py -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $D/pytest.log
[ $rc -ne 0 ] && exit 1
HB2ST_PROBE_NOHOST=1 timeout -k 10 200 python -u tools/probe/hb2st_time.py 16384 64 > $D/hb2st.log 2>&1 || { tail $D/hb2st.log; exit 1; }
cat $D/hb2st.log
timeout -k 10 300 python -u bench.py --routine heev --n 16384 --nb 256 --steps 2 --warmup 1 > $D/bench_heev.log 2>&1 || { tail $D/bench_heev.log; exit 1; }
tail -1 $D/bench_heev.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof_getrf -o run -- python3 $GRAFT_REPO_ROOT/bench.py --routine getrf --lookahead 2 --steps 1 --warmup 1 > $GRAFT_REPO_ROOT/$D/prof_getrf.log 2>&1 || { tail $GRAFT_REPO_ROOT/$D/prof_getrf.log; exit 1; }
grep metric $GRAFT_REPO_ROOT/$D/prof_getrf.log | cut -c1-160
