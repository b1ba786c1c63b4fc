#!/bin/bash
# bench input restore: overlapped double buffer vs inline copy
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/restore
for r in potrf getrf geqrf; do
  extra=""; [ $r = geqrf ] && extra="--m 65536 --n 8192 --nb 256"; [ $r = getrf ] && extra="--lookahead 2"
  for mode in overlap inline; do
    SLATE_AMD_BENCH_RESTORE=$mode timeout -k 10 200 python -u bench.py --routine $r $extra --steps 5 --warmup 2 > gpurun_out/restore/${r}_$mode.log 2>&1 || { tail gpurun_out/restore/${r}_$mode.log; exit 1; }
    echo "$r $mode: $(grep -o '"value": [0-9.]*\|"residual": [0-9.e-]*\|"info_ok": [a-z]*' gpurun_out/restore/${r}_$mode.log | tr '\n' ' ')"
  done
done
