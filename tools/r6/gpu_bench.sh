#!/bin/bash
# headline bench (driver contract) + smoke + rocprof stats of the bench
set -o pipefail
mkdir -p gpurun_out/r6/bench
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6/bench/smoke.log 2>&1 || { tail -5 gpurun_out/r6/bench/smoke.log; exit 1; }
tail -2 gpurun_out/r6/bench/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r6/bench/bench.json 2> gpurun_out/r6/bench/bench.err || { tail -5 gpurun_out/r6/bench/bench.err; exit 1; }
cat gpurun_out/r6/bench/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r6/bench/prof -o potrf -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r6/bench/prof.log 2>&1
echo "rocprof rc=$?"
