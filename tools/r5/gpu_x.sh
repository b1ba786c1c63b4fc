#!/bin/bash
# recursive panel trsm: numerics, dpotrf (python + native) with it on / off, 2x4 loopback
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/x; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "trsm or potrf or chol" --timeout 240 --timeout-method thread > $D/tests.log 2>&1
rc=$?; tail -2 $D/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $D/tests.log | head; exit 1; }
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("residual"))'; }
for rec in 1 0 1; do
  SLATE_AMD_TRSM_RLT_REC=$rec timeout -k 10 200 python -u bench.py > $D/potrf_rec$rec.log 2>&1 || { tail -3 $D/potrf_rec$rec.log; exit 1; }
  echo "potrf rec=$rec: $(tail -1 $D/potrf_rec$rec.log | j)"
done
SLATE_AMD_TRSM_RLT_REC=1 timeout -k 10 200 python -u bench.py --impl native > $D/npotrf.log 2>&1 || { tail -3 $D/npotrf.log; exit 1; }
echo "native potrf: $(tail -1 $D/npotrf.log | j)"
timeout -k 10 300 python -u tools/r5/loopback_critpath.py --routine potrf --ranks 0,5 > $D/lb.log 2>&1 || { tail -5 $D/lb.log; exit 1; }
grep "Job projection" $D/lb.log; grep -E '^\| [05] ' $D/lb.log
