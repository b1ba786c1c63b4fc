#!/bin/bash
# quick knob sweep: LU deferred left-swap tail fraction; stage-1 back-transform group size
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${TAG:-s24}; mkdir -p $D
for f in 0.4 0.8; do
  SLATE_AMD_LU_LEFT_TAIL=$f timeout -k 10 200 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 > $D/b.log 2>&1 || { tail -3 $D/b.log; exit 1; }
  echo "left_tail $f: $(tail -1 $D/b.log | grep -o '"value": [0-9.]*') $(tail -1 $D/b.log | grep -o '"residual_ok": [a-z]*')"
done
for g in 8 2; do
  SLATE_AMD_UNMTR_HE2HB_GROUP=$g timeout -k 10 300 python -u tools/heev_phases.py 16384 256 > $D/h.log 2>&1 || { tail -3 $D/h.log; exit 1; }
  echo "he2hb group $g: $(grep 'heev n=' $D/h.log) | $(grep 'device   unmtr_he2hb' $D/h.log)"
done
