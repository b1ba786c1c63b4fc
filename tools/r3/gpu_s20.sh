#!/bin/bash
# dgetrf sweep with the current panel kernel: rows-per-thread threshold x reserved panel CUs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${TAG:-s20}; mkdir -p $D
for cfg in "SLATE_AMD_LU_RPT1_ROWS=16384 SLATE_AMD_PANEL_CUS=32" "SLATE_AMD_LU_RPT1_ROWS=24576 SLATE_AMD_PANEL_CUS=48" "SLATE_AMD_LU_RPT1_ROWS=16384 SLATE_AMD_PANEL_CUS=24" "SLATE_AMD_LU_RPT1_ROWS=16384 SLATE_AMD_PANEL_CUS=40" "SLATE_AMD_LU_RPT1_ROWS=8192 SLATE_AMD_PANEL_CUS=32"; do
  env $cfg timeout -k 10 200 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 > $D/b.log 2>&1 || { echo "$cfg failed"; tail -3 $D/b.log; exit 1; }
  echo "$cfg: $(tail -1 $D/b.log | grep -o '"value": [0-9.]*') $(tail -1 $D/b.log | grep -o '"residual_ok": [a-z]*')"
done
