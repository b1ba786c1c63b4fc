#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6/ae
for r in getrf potrf; do
  timeout -k 10 300 python -u bench.py --impl native --routine $r --steps 3 --warmup 1 > gpurun_out/r6/ae/$r.json 2>/dev/null || exit 1
  echo "$r $(python -c "import json;d=json.load(open('gpurun_out/r6/ae/$r.json'));print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_native_gpu.py > gpurun_out/r6/ae/native.log 2>&1
rc=$?
tail -2 gpurun_out/r6/ae/native.log
exit $rc
