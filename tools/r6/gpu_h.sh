#!/bin/bash
# kernel trace of the 1-GPU dgetrf bench (Python driver and native driver):
# update-stream gaps and per-stream kernel time
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r6/h; mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/getrf -o run -- python3 bench.py --routine getrf --steps 2 --warmup 1 > $D/getrf.log 2>&1
rc=$?; tail -1 $D/getrf.log; [ $rc -eq 0 ] || exit $rc
f=$(find $D/getrf -name '*kernel_trace.csv' | head -1)
python3 tools/r6/potrf_gaps.py $f > $D/getrf_gaps.txt 2>&1; cat $D/getrf_gaps.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/ngetrf -o run -- python3 bench.py --impl native --routine getrf --steps 2 --warmup 1 > $D/ngetrf.log 2>&1
rc=$?; tail -1 $D/ngetrf.log; [ $rc -eq 0 ] || exit $rc
f=$(find $D/ngetrf -name '*kernel_trace.csv' | head -1)
python3 tools/r6/potrf_gaps.py $f > $D/ngetrf_gaps.txt 2>&1; cat $D/ngetrf_gaps.txt
find $D -name "*.csv" -size +40M -delete
exit 0
