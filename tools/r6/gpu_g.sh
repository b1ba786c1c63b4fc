#!/bin/bash
# one-rank dpotrf n=32768: head / tail one-tile groups, group size, lookahead
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6/g; mkdir -p $D
out=$D/potrf_schedule_sweep.txt; : > $out
for cfg in "0 0 2 1" "1 0 2 1" "0 4 2 1" "0 8 2 1" "1 8 2 1" "0 16 2 1" "0 0 3 1" "0 0 4 1" "0 8 3 1" "0 0 2 2" "0 8 2 2"; do
  set -- $cfg
  r=$(SLATE_AMD_POTRF_HEAD=$1 SLATE_AMD_POTRF_TAIL=$2 SLATE_AMD_POTRF_GROUP=$3 timeout -k 10 120 python bench.py --steps 6 --warmup 2 --lookahead $4 2>/dev/null | grep '^{')
  rc=$?; [ $rc -eq 0 ] || { echo "fail $cfg rc=$rc" >> $out; exit $rc; }
  echo "head $1 tail $2 group $3 la $4: $(echo $r | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], "ms", d["value"], "GF/s", d["residual_ok"])')" | tee -a $out
done
