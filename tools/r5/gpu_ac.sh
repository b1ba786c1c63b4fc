#!/bin/bash
# masked-GEMM block order: row-interleaved XCD chunks (3) vs plain order (0), 2x4 loopback dpotrf + GEMM tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/ac; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm or herk or syrk or mask" --timeout 240 --timeout-method thread > $D/tests.log 2>&1
rc=$?; tail -2 $D/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $D/tests.log | head; exit 1; }
for r in 3 0 3; do
  SLATE_AMD_GEMM_MASK_REMAP=$r timeout -k 10 300 python -u tools/r5/loopback_critpath.py --routine potrf --ranks 0,5 > $D/lb_$r.log 2>&1 || { tail -5 $D/lb_$r.log; exit 1; }
  echo "remap $r: $(grep -E '^\| [05] ' $D/lb_$r.log | awk -F'|' '{printf "r%s loopback %s proj %s; ", $2, $4, $7}')"
done
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 > $D/potrf.log 2>&1 || { tail -3 $D/potrf.log; exit 1; }
echo "1-GPU potrf: $(tail -1 $D/potrf.log | j)"
