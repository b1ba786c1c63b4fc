#!/bin/bash
# round 5 / c: peer-mailbox LU panel (2 / 4 ranks on one GPU), native tests
# (ScaLAPACK sub-matrices, p?trsm_ Right / complex T, native peer panel), GEMM sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5; mkdir -p $D
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_dist_gpu.py -k "peer_mailbox or multirank" > $D/pytest_c1.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error|peer LU stats|passed|failed" $D/pytest_c1.log | tail -30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_native_gpu.py > $D/pytest_c2.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed" $D/pytest_c2.log | tail -20; [ $rc -ne 0 ] && { tail -60 $D/pytest_c2.log; exit $rc; }
timeout -k 10 200 ./tools/exp/gemm_sweep_r5.bin > $D/gemm_sweep.txt 2>&1 || { cat $D/gemm_sweep.txt; exit 1; }
cat $D/gemm_sweep.txt
