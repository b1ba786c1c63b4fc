#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/v; mkdir -p $D
timeout -k 10 120 ./slate_amd/ex_native 1x1 > $D/ex11.log 2>&1; rc=$?
grep -E "check (trtri|trtrm|gesv_nopiv|cholqr|gelqf)_" $D/ex11.log; [ $rc -ne 0 ] && { tail -5 $D/ex11.log; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_native_gpu.py -x -q --timeout 240 --timeout-method thread > $D/native.log 2>&1
rc=$?; tail -3 $D/native.log; [ $rc -ne 0 ] && { grep -E "assert|Error" $D/native.log | head -10; exit 1; }
exit 0
