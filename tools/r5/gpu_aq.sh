#!/bin/bash
# in-DAG link model: spin sanity, then 2x4 / 2x2 / 2x1 potrf projections
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/aq; mkdir -p $D
timeout -k 10 120 python3 -c "
import torch, time
from slate_amd import ops
x = torch.zeros(1, device='cuda')
ops.spin_ns(1e5, x); torch.cuda.synchronize()
for ns in (1e5, 1e6, 1e7):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); ops.spin_ns(ns, x); e1.record(); torch.cuda.synchronize()
    print('spin', ns / 1e6, 'ms requested ->', round(e0.elapsed_time(e1), 3), 'ms')
" > $D/spin.log 2>&1 || { cat $D/spin.log; exit 1; }
grep spin $D/spin.log
for L in 10,150 25,50; do
  for la in 1 2; do
    timeout -k 10 200 python3 tools/r5/loopback_critpath.py --grid 2x4 --ranks 0,5 --lookahead $la --link $L > $D/lb_2x4_la${la}_$L.log 2>&1 || exit $?
    grep -h "job" $D/lb_2x4_la${la}_$L.log | sed "s/^/2x4 la=$la link=$L /"
  done
  for g in 2x2 2x1 1x2; do
    timeout -k 10 200 python3 tools/r5/loopback_critpath.py --grid $g --ranks 0 --link $L > $D/lb_${g}_$L.log 2>&1 || exit $?
    grep -h "job" $D/lb_${g}_$L.log | sed "s/^/$g la=1 link=$L /"
  done
done
