#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5; mkdir -p $D
EX_NATIVE_TYPES=d SLATE_AMD_NATIVE_HEEV_DEBUG=1 timeout -k 10 240 ./slate_amd/ex_native 1x1 > $D/ex_native_dbg.txt 2>&1; rc=$?
grep -E "heev|check (heev|gecondest)" $D/ex_native_dbg.txt; exit $rc
