#!/bin/bash
# round 5 / e: native tests (heev, condest, ScaLAPACK sub-matrices), peer LU timing rehearsal, GEMM sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5; mkdir -p $D
timeout -k 10 240 ./slate_amd/ex_native 1x1 > $D/ex_native_1x1.txt 2>&1; rc=$?
grep -E "check (heev|gecondest)" $D/ex_native_1x1.txt; [ $rc -ne 0 ] && { tail -30 $D/ex_native_1x1.txt; exit $rc; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_native_gpu.py > $D/pytest_e.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed" $D/pytest_e.log | tail -20; [ $rc -ne 0 ] && { grep -E "check r|Error|error" $D/pytest_e.log | head -60; exit $rc; }
timeout -k 10 300 python -u tools/probe/lu_peer_time.py 8192 512 > $D/lu_peer_time.txt 2>&1; rc=$?; tail -8 $D/lu_peer_time.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 ./tools/exp/gemm_sweep_r5.bin > $D/gemm_sweep.txt 2>&1 || { cat $D/gemm_sweep.txt; exit 1; }
cat $D/gemm_sweep.txt
