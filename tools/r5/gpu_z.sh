#!/bin/bash
# dgetrf knob sweep after the glds GEMM (one MI355X), and the dsyevd band width
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/z; mkdir -p $D
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for cfg in "0 0.6" "0.25 0.6" "0.5 0.6" "0 0.8" "0 0.4" "0.25 0.8"; do
  set -- $cfg
  SLATE_AMD_LU_UNMASKED=$1 SLATE_AMD_LU_LEFT_TAIL=$2 timeout -k 10 200 python -u bench.py --routine getrf --lookahead 2 --steps 2 --warmup 1 --check 0 > $D/g_$1_$2.log 2>&1 || { tail -3 $D/g_$1_$2.log; exit 1; }
  echo "getrf unmasked $1 left_tail $2: $(tail -1 $D/g_$1_$2.log | j)"
done
for b in 32 48 64 96; do
  timeout -k 10 200 python -u bench.py --routine heev --n 16384 --nb 256 --band $b --steps 1 --warmup 1 --check 0 > $D/h_$b.log 2>&1 || { tail -3 $D/h_$b.log; exit 1; }
  echo "heev band $b: $(tail -1 $D/h_$b.log | j)"
done
