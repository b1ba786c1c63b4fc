#!/bin/bash
# chase: progress flags in uncached memory vs the caller's (cached) buffer
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for f in cached uncached; do
  SLATE_AMD_HB2ST_FLAGS=$f timeout -k 10 200 python -u tools/probe/hb2st_time.py 16384 64 > gpurun_out/hb2st_flags_$f.log 2>&1 || { tail gpurun_out/hb2st_flags_$f.log; exit 1; }
  echo "flags=$f: $(grep -h 'device\|phases\|eig diff' gpurun_out/hb2st_flags_$f.log | tr '\n' ' ')"
done
