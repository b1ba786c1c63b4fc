#!/bin/bash
# 64x64-tile trailing GEMMs in the distributed potrf (shorter workgroups)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/bd; mkdir -p $D
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "stair or trimask" > $D/kt.log 2>&1 || { tail -20 $D/kt.log; exit 1; }
SLATE_AMD_GEMM_TILE64=1 timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "stair or trimask or gemm" >> $D/kt.log 2>&1 || { tail -20 $D/kt.log; exit 1; }
grep passed $D/kt.log
for L in 10,150 25,50; do
  for t in 0 1; do
    SLATE_AMD_GEMM_TILE64=$t timeout -k 10 200 python3 tools/r5/loopback_critpath.py --grid 2x4 --ranks 0,5 --link $L > $D/lb_${t}_$L.log 2>&1 || exit $?
    grep -h "job" $D/lb_${t}_$L.log | sed "s/^/2x4 tile64=$t link=$L /"
  done
done
SLATE_AMD_GEMM_TILE64=1 timeout -k 10 200 python3 tools/r5/loopback_critpath.py --grid 2x2 --ranks 0 --link 10,150 > $D/lb22.log 2>&1 || exit $?
grep -h "job" $D/lb22.log | sed "s/^/2x2 tile64=1 link=10,150 /"
