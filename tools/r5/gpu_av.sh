#!/bin/bash
# 2x4 potrf under the in-DAG link model: diag-tile kernel, lookahead, chunking
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/av; mkdir -p $D
run() {  # name, env..., then args
  local name=$1; shift
  env "$@" timeout -k 10 200 python3 tools/r5/loopback_critpath.py --grid 2x4 --ranks 0,5 --link $L $XA > $D/lb_${name}_$L.log 2>&1 || exit $?
  grep -h "job" $D/lb_${name}_$L.log | sed "s/^/2x4 $name link=$L /"
}
for L in 10,150 25,50; do
  XA="" run base SLATE_AMD_X=0
  XA="" run lds SLATE_AMD_POTRF_TILE=lds
  XA="--lookahead 2" run la2 SLATE_AMD_X=0
  XA="" run ch8 SLATE_AMD_POTRF_CHUNK=8
  XA="" run ch16 SLATE_AMD_POTRF_CHUNK=16
  XA="" run nodf SLATE_AMD_POTRF_DIAGFIRST=0
done
