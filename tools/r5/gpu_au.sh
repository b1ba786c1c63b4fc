#!/bin/bash
# auto trsm K split: kernel tests, 2x4 link projections, 1-GPU potrf bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/au; mkdir -p $D
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "trsm or potrf" > $D/kt.log 2>&1 || { tail -30 $D/kt.log; exit 1; }
tail -1 $D/kt.log
for L in 10,150 25,50; do
  timeout -k 10 200 python3 tools/r5/loopback_critpath.py --grid 2x4 --ranks 0,5 --link $L > $D/lb_$L.log 2>&1 || exit $?
  grep -h "job" $D/lb_$L.log | sed "s/^/2x4 auto-ks link=$L /"
  SLATE_AMD_TRSM_KS=1 timeout -k 10 200 python3 tools/r5/loopback_critpath.py --grid 2x4 --ranks 0,5 --link $L > $D/lb1_$L.log 2>&1 || exit $?
  grep -h "job" $D/lb1_$L.log | sed "s/^/2x4 ks=1 link=$L /"
done
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 > $D/bench.json 2> $D/bench.err || { tail $D/bench.err; exit 1; }
cat $D/bench.json
SLATE_AMD_TRSM_KS=1 timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 > $D/bench1.json 2> $D/bench1.err || { tail $D/bench1.err; exit 1; }
cat $D/bench1.json
