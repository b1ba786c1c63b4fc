#!/bin/bash
# trailing column gather on the update stream (col_comm_u) + chunk 16
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/ax; mkdir -p $D
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_nosync_gpu.py tests/test_loopback.py tests/test_dist_gpu.py > $D/t.log 2>&1 || { tail -30 $D/t.log; exit 1; }
tail -1 $D/t.log
for L in 10,150 25,50; do
  for u in 1 0; do
    SLATE_AMD_POTRF_LCOL_U=$u timeout -k 10 200 python3 tools/r5/loopback_critpath.py --grid 2x4 --ranks 0,5 --link $L > $D/lb_u${u}_$L.log 2>&1 || exit $?
    grep -h "job" $D/lb_u${u}_$L.log | sed "s/^/2x4 lcol_u=$u link=$L /"
  done
  timeout -k 10 200 python3 tools/r5/loopback_critpath.py --grid 2x2 --ranks 0 --link $L > $D/lb22_$L.log 2>&1 || exit $?
  grep -h "job" $D/lb22_$L.log | sed "s/^/2x2 link=$L /"
  timeout -k 10 200 python3 tools/r5/loopback_critpath.py --grid 2x1 --ranks 0 --link $L > $D/lb21_$L.log 2>&1 || exit $?
  grep -h "job" $D/lb21_$L.log | sed "s/^/2x1 link=$L /"
  timeout -k 10 200 python3 tools/r5/loopback_critpath.py --grid 1x2 --ranks 0 --link $L > $D/lb12_$L.log 2>&1 || exit $?
  grep -h "job" $D/lb12_$L.log | sed "s/^/1x2 link=$L /"
done
