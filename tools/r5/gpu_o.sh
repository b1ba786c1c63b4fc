#!/bin/bash
# knob sweep after the glds GEMM: potrf group size x lookahead, getrf lookahead
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/o; mkdir -p $D
for g in 1 2 3 4; do for la in 1 2; do
  SLATE_AMD_POTRF_GROUP=$g timeout -k 10 120 python -u bench.py --lookahead $la --steps 3 --warmup 1 --check 0 > $D/potrf_g${g}_la${la}.log 2>&1 || { tail -3 $D/potrf_g${g}_la${la}.log; exit 1; }
  echo "potrf group $g lookahead $la: $(tail -1 $D/potrf_g${g}_la${la}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
for la in 1 2 3; do
  timeout -k 10 120 python -u bench.py --routine getrf --lookahead $la --steps 2 --warmup 1 --check 0 > $D/getrf_la${la}.log 2>&1 || { tail -3 $D/getrf_la${la}.log; exit 1; }
  echo "getrf lookahead $la: $(tail -1 $D/getrf_la${la}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
