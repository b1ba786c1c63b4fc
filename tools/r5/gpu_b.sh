#!/bin/bash
# round 5 / b: GEMM tile sweep, peer-mailbox LU panel tests (2 and 4 ranks on one GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5; mkdir -p $D
timeout -k 10 200 ./tools/exp/gemm_sweep_r5.bin > $D/gemm_sweep.txt 2>&1 || { cat $D/gemm_sweep.txt; exit 1; }
cat $D/gemm_sweep.txt
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_dist_gpu.py -k "peer_mailbox or multirank" > $D/pytest_b.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error|peer LU stats|passed|failed" $D/pytest_b.log | tail -30; exit $rc
