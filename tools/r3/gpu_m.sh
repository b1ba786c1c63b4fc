#!/bin/bash
# unmtr_hb2st Z-window pitch + hb2st pitch 4 (default now): dsyevd n=16384, and the eig GPU tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && export PYTHONPATH="$GRAFT_REPO_ROOT"
O=gpurun_out/r3m
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_eig_svd.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_eig.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_eig.log
[ $rc -ne 0 ] && exit 1
for it in 1 2; do
  timeout -k 10 240 python -u bench.py --routine heev --n 16384 --nb 256 --steps 1 --warmup 1 > $O/heev_$it.log 2>&1 || { echo "heev failed"; tail -5 $O/heev_$it.log; exit 1; }
  tail -1 $O/heev_$it.log
done
