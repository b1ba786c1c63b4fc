#!/bin/bash
# native vs Python dgetrf n=32768: lookahead 1/2 and kernel stats
set -o pipefail
mkdir -p gpurun_out/r6/ab
for la in 1 2; do
  timeout -k 10 300 python -u bench.py --impl native --routine getrf --steps 3 --warmup 1 --lookahead $la > gpurun_out/r6/ab/native_la$la.json 2>/dev/null || exit 1
  echo "native la=$la $(python -c "import json;d=json.load(open('gpurun_out/r6/ab/native_la$la.json'));print(d['value'], d['ms_per_step'])")"
  timeout -k 10 300 python -u bench.py --routine getrf --steps 3 --warmup 1 --lookahead $la > gpurun_out/r6/ab/py_la$la.json 2>/dev/null || exit 1
  echo "python la=$la $(python -c "import json;d=json.load(open('gpurun_out/r6/ab/py_la$la.json'));print(d['value'], d['ms_per_step'])")"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r6/ab/prof_native -o run -- $GRAFT_REPO_ROOT/slate_amd/bench_native getrf 32768 512 1 1 2 1 2 0 > $GRAFT_REPO_ROOT/gpurun_out/r6/ab/prof_native.log 2>&1
echo "rocprof native rc=$?"
