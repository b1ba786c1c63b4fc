#!/bin/bash
# dgetrf: trailing updates of the first steps on all CUs (SLATE_AMD_LU_UNMASKED sweep)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${TAG:-s5}; mkdir -p $D
for f in 0 0.2 0.35 0.5; do
  SLATE_AMD_LU_UNMASKED=$f timeout -k 10 200 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 > $D/bench_getrf_$f.log 2>&1 || { tail $D/bench_getrf_$f.log; exit 1; }
  echo "unmasked $f: $(tail -1 $D/bench_getrf_$f.log | cut -c1-150)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof_heev -o run -- python3 $GRAFT_REPO_ROOT/bench.py --routine heev --n 16384 --nb 256 --steps 1 --warmup 0 > $GRAFT_REPO_ROOT/$D/prof_heev.log 2>&1 || { tail $GRAFT_REPO_ROOT/$D/prof_heev.log; exit 1; }
tail -1 $GRAFT_REPO_ROOT/$D/prof_heev.log
