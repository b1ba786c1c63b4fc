#!/bin/bash
# round 5 / g: GEMM prefetch-depth experiment, native tests (svd added)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5; mkdir -p $D
timeout -k 10 240 ./slate_amd/ex_native 1x1 > $D/ex_native_1x1.txt 2>&1; rc=$?
grep -E "check (heev|svd|gecondest)" $D/ex_native_1x1.txt; [ $rc -ne 0 ] && { tail -30 $D/ex_native_1x1.txt; exit $rc; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_native_gpu.py > $D/pytest_g.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed" $D/pytest_g.log | tail -20; [ $rc -ne 0 ] && { grep -E "check r|Error|error" $D/pytest_g.log | head -60; exit $rc; }
timeout -k 10 300 ./tools/exp/gemm_pf_r5.bin > $D/gemm_pf.txt 2>&1 || { cat $D/gemm_pf.txt; exit 1; }
cat $D/gemm_pf.txt
