#!/bin/bash
# staircase-compacted masked GEMM: numerics (kernel + driver tests), isolated probe on / off, 2x4 loopback, 1-GPU potrf
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/ag; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_dist_gpu.py -x -q --timeout 240 --timeout-method thread > $D/tests.log 2>&1
rc=$?; tail -2 $D/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $D/tests.log | head; exit 1; }
for st in 1 0; do echo "stair $st:"; SLATE_AMD_GEMM_STAIR=$st timeout -k 10 120 python3 tools/r5/masked_gemm_probe.py 2>&1 | grep -E "masked|rectangle" || exit 1; done
for st in 1 0; do
  SLATE_AMD_GEMM_STAIR=$st timeout -k 10 300 python -u tools/r5/loopback_critpath.py --routine potrf --ranks 0,5 > $D/lb_$st.log 2>&1 || { tail -5 $D/lb_$st.log; exit 1; }
  echo "stair $st: $(grep -E '^\| [05] ' $D/lb_$st.log | awk -F'|' '{printf "r%s loopback %s proj %s; ", $2, $4, $7}')"
done
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["residual"])'; }
timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 > $D/potrf.log 2>&1 || { tail -3 $D/potrf.log; exit 1; }
echo "1-GPU potrf: $(tail -1 $D/potrf.log | j)"
