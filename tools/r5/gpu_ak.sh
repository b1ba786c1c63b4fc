#!/bin/bash
# eig / svd GPU tests (single + distributed over gloo on one GPU) after the device band assembly
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/ak; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_native_gpu.py tests -m gpu -x -q -k "native or svd or heev or eig or band or census" --timeout 300 --timeout-method thread > $D/tests.log 2>&1
rc=$?; tail -3 $D/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $D/tests.log | head; exit 1; }

j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["metric"], d["value"], d.get("ms_per_step"), d.get("residual"))'; }
timeout -k 10 300 python -u bench.py --routine geqrf --m 65536 --n 8192 --steps 3 --warmup 1 > $D/geqrf.log 2>&1 || { tail -3 $D/geqrf.log; exit 1; }
echo "geqrf: $(tail -1 $D/geqrf.log | j)"
timeout -k 10 300 python -u bench.py --impl native --routine geqrf --m 65536 --n 8192 --steps 3 --warmup 1 > $D/ngeqrf.log 2>&1 || { tail -3 $D/ngeqrf.log; exit 1; }
echo "native geqrf: $(tail -1 $D/ngeqrf.log | j)"
