#!/bin/bash
# full GPU suite + smoke + potrf / getrf benches on the current tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/${TAG:-full}; mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $D/pytest.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error" $D/pytest.log | head -20; exit 1; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 200 python -u bench.py > $D/bench_potrf.log 2>&1 || { tail $D/bench_potrf.log; exit 1; }
tail -1 $D/bench_potrf.log
timeout -k 10 200 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 > $D/bench_getrf.log 2>&1 || { tail $D/bench_getrf.log; exit 1; }
tail -1 $D/bench_getrf.log
