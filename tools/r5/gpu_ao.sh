#!/bin/bash
# stair mapping rewrite + potrf step pairs: tests, probe, loopback projections
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/ao; mkdir -p $D
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "trimask or stair or gemm" > $D/kt.log 2>&1 || { tail -30 $D/kt.log; exit 1; }
tail -1 $D/kt.log
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_nosync_gpu.py > $D/ns.log 2>&1 || { tail -30 $D/ns.log; exit 1; }
tail -1 $D/ns.log
for g in 1x1 1x2 2x1 2x4; do
  timeout -k 10 120 python3 tools/r5/stair_probe.py --grid $g >> $D/probe.log 2>&1 || exit $?
done
grep -v amdgpu.ids $D/probe.log
for g in 1x2 2x1 2x2; do
  timeout -k 10 200 python3 tools/r5/loopback_critpath.py --grid $g --ranks 0 > $D/lb_$g.log 2>&1 || exit $?
  grep "Job projection" $D/lb_$g.log
done
timeout -k 10 200 python3 tools/r5/loopback_critpath.py --grid 2x4 --ranks 0,1,5 > $D/lb_2x4.log 2>&1 || exit $?
grep "Job projection" $D/lb_2x4.log
SLATE_AMD_POTRF_PAIR=0 timeout -k 10 200 python3 tools/r5/loopback_critpath.py --grid 2x4 --ranks 0,1,5 > $D/lb_2x4_nopair.log 2>&1 || exit $?
grep "Job projection" $D/lb_2x4_nopair.log
