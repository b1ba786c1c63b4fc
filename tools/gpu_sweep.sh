#!/bin/bash
# potrf / getrf knob sweep: reserved panel CUs x lookahead
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/sweep.log; : > $out
for r in ${ROUTINES:-potrf}; do
for cus in ${CUS:-0 16 32 64}; do for la in ${LAS:-1 2}; do
  echo "routine=$r cus=$cus la=$la" >> $out
  SLATE_AMD_PANEL_CUS=$cus timeout -k 10 120 python -u bench.py --routine $r --lookahead $la --steps 2 --warmup 1 --check 0 2>&1 | grep -o '"value": [^,]*' >> $out || exit 1
done; done; done
