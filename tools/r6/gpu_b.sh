#!/bin/bash
# kernel trace of the 1-GPU dpotrf bench: update-stream gaps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r6/b; mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/bench -o run -- python3 bench.py --steps 2 --warmup 1 > $D/bench.log 2>&1
rc=$?; tail -2 $D/bench.log; [ $rc -eq 0 ] || exit $rc
f=$(find $D/bench -name '*kernel_trace.csv' | head -1)
python3 tools/r6/potrf_gaps.py $f > $D/gaps.txt 2>&1; cat $D/gaps.txt
