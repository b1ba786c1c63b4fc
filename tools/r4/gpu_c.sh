#!/bin/bash
# native first-call probe (NaN-poisoned scratch) + stedc device merges
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/r4/scal_repro.py 1 > gpurun_out/scal_repro.log 2>&1; echo "scal rc=$?"
grep -E "iter|rep" gpurun_out/scal_repro.log | head -20
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_eig_svd.py -m gpu -k "stedc or heev or syev" > gpurun_out/stedc.log 2>&1; echo "stedc rc=$?"
grep -E "PASSED|FAILED|Error|assert" gpurun_out/stedc.log | head -40
