#!/bin/bash
# 2x4 loopback dpotrf knob sweep: row-broadcast chunking, lookahead, diag-first
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/r; mkdir -p $D
for cfg in "4 1 1" "2 1 1" "8 1 1" "16 1 1" "4 2 1" "4 1 0" "8 2 1"; do
  set -- $cfg
  SLATE_AMD_POTRF_CHUNK=$1 SLATE_AMD_POTRF_DIAGFIRST=$3 timeout -k 10 200 python -u tools/r5/loopback_critpath.py --routine potrf --ranks 0,5 --lookahead $2 > $D/c$1_la$2_df$3.log 2>&1 || { tail -5 $D/c$1_la$2_df$3.log; exit 1; }
  echo "chunk $1 la $2 diagfirst $3: $(grep -E '^\| [05] ' $D/c$1_la$2_df$3.log | awk -F'|' '{printf "r%s loopback %s proj %s; ", $2, $4, $7}')"
done
