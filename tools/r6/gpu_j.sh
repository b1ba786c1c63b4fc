#!/bin/bash
# one-rank dgetrf n=32768: reserved panel CUs, unmasked GEMM-bound head, lookahead
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6/j; mkdir -p $D
out=$D/getrf_sweep.txt; : > $out
for cfg in "32 0 1" "64 0 1" "96 0 1" "128 0 1" "32 0.5 1" "64 0.5 1" "64 0.6 1" "32 0 2" "64 0 2"; do
  set -- $cfg
  r=$(SLATE_AMD_PANEL_CUS=$1 SLATE_AMD_LU_UNMASKED=$2 timeout -k 10 150 python bench.py --routine getrf --steps 3 --warmup 1 --lookahead $3 2>/dev/null | grep '^{')
  rc=$?; [ $rc -eq 0 ] || { echo "fail $cfg rc=$rc" >> $out; exit $rc; }
  echo "cus $1 unmasked $2 la $3: $(echo $r | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], "ms", d["value"], "GF/s", d["residual_ok"])')" | tee -a $out
done
