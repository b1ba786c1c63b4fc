#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/ay; mkdir -p $D
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm" > $D/kt.log 2>&1 || { tail -20 $D/kt.log; exit 1; }
SLATE_AMD_GEMM_SOLO=1 timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm" >> $D/kt.log 2>&1 || { tail -20 $D/kt.log; exit 1; }
grep passed $D/kt.log
for L in 10,150 25,50; do
  for so in 0 1; do
    SLATE_AMD_GEMM_SOLO=$so timeout -k 10 200 python3 tools/r5/loopback_critpath.py --grid 2x4 --ranks 0,5 --link $L > $D/lb_$so_$L.log 2>&1 || exit $?
    grep -h "job" $D/lb_$so_$L.log | sed "s/^/2x4 solo=$so link=$L /"
  done
done
SLATE_AMD_GEMM_SOLO=1 timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 > $D/bench_solo.json 2> $D/bench.err || { tail $D/bench.err; exit 1; }
cat $D/bench_solo.json
