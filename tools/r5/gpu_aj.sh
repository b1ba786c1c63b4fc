#!/bin/bash
# 2x4 loopback dpotrf: tile Cholesky kernel choice (multi-workgroup mc vs one-CU lds)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/aj; mkdir -p $D
for t in mc lds mc; do
  SLATE_AMD_POTRF_TILE=$t timeout -k 10 300 python -u tools/r5/loopback_critpath.py --routine potrf --ranks 0,5 > $D/lb_$t.log 2>&1 || { tail -5 $D/lb_$t.log; exit 1; }
  echo "tile $t: $(grep -E '^\| [05] ' $D/lb_$t.log | awk -F'|' '{printf "r%s loopback %s proj %s; ", $2, $4, $7}')"
done
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for t in lds mc; do
  SLATE_AMD_POTRF_TILE=$t timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --check 0 > $D/p_$t.log 2>&1 || { tail -3 $D/p_$t.log; exit 1; }
  echo "1-GPU potrf tile $t: $(tail -1 $D/p_$t.log | j)"
done
