#!/bin/bash
# the other 1-GPU benches after the glds GEMM: geqrf, heev (dsyevd n=16384), gemm, native potrf/getrf/geqrf
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/t; mkdir -p $D
run() { local name=$1; shift; timeout -k 10 300 python -u bench.py "$@" > $D/$name.log 2>&1 || { tail -5 $D/$name.log; exit 1; }; echo "$name: $(tail -1 $D/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["metric"], d["value"], d["unit"], d.get("ms_per_step"))')"; }
run geqrf --routine geqrf --steps 3 --warmup 1
run heev --routine heev --n 16384 --nb 256 --steps 2 --warmup 1
run potrf_native --impl native --steps 3 --warmup 1
run getrf_native --impl native --routine getrf --lookahead 2 --steps 3 --warmup 1
run geqrf_native --impl native --routine geqrf --steps 3 --warmup 1
