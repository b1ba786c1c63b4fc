#!/bin/bash
# loopback projection of the 2x4 dpotrf / dgemm critical path (one GPU plays ranks of the 8-GPU job)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/p; mkdir -p $D
rm -f $D/critpath_2x4.md
timeout -k 10 300 python -u tools/r5/loopback_critpath.py --routine potrf --ranks 0,1,5 --out $D/critpath_2x4.md > $D/potrf.log 2>&1 || { tail -20 $D/potrf.log; exit 1; }
grep -A8 "^| rank" $D/potrf.log | head -12
timeout -k 10 300 python -u tools/r5/loopback_critpath.py --routine potrf --ranks 0,5 --lookahead 2 --out $D/critpath_2x4.md > $D/potrf_la2.log 2>&1 || { tail -20 $D/potrf_la2.log; exit 1; }
grep "Job projection" $D/potrf_la2.log
timeout -k 10 300 python -u tools/r5/loopback_critpath.py --routine gemm --ranks 0,5 --out $D/critpath_2x4.md > $D/gemm.log 2>&1 || { tail -20 $D/gemm.log; exit 1; }
grep "Job projection" $D/gemm.log
