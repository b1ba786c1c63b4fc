#!/bin/bash
# round 5 / d: native tests (ScaLAPACK sub-matrices), peer LU timing rehearsal, GEMM sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5; mkdir -p $D
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_native_gpu.py > $D/pytest_d.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed" $D/pytest_d.log | tail -20; [ $rc -ne 0 ] && { grep -E "check r|Error" $D/pytest_d.log | head -60; exit $rc; }
timeout -k 10 300 python -u tools/probe/lu_peer_time.py 8192 512 > $D/lu_peer_time.txt 2>&1; rc=$?; cat $D/lu_peer_time.txt | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 ./tools/exp/gemm_sweep_r5.bin > $D/gemm_sweep.txt 2>&1 || { cat $D/gemm_sweep.txt; exit 1; }
cat $D/gemm_sweep.txt
