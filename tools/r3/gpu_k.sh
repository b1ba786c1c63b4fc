#!/bin/bash
# full GPU test suite + smoke + headline bench (round-end rehearsal)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && export PYTHONPATH="$GRAFT_REPO_ROOT"
O=gpurun_out/r3k
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 200 python -u bench.py > $O/bench.log 2>&1 || { echo bench failed; tail $O/bench.log; exit 1; }
tail -1 $O/bench.log
