#!/bin/bash
# unmtr_hb2st with precomputed V^T fragments: eig GPU tests, heev phases + bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${TAG:-s23}; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_eig_svd.py -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $D/pytest.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python -u tools/heev_phases.py 16384 256 > $D/heev_phases.log 2>&1 || { tail $D/heev_phases.log; exit 1; }
cat $D/heev_phases.log
timeout -k 10 300 python -u bench.py --routine heev --n 16384 --nb 256 --steps 2 --warmup 1 > $D/bench_heev.log 2>&1 || { tail $D/bench_heev.log; exit 1; }
tail -1 $D/bench_heev.log | cut -c1-150
