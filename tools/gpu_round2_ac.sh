#!/bin/bash
# bulge chase: LDS staging size sweep + phase split; tb2bd timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for kb in 96 128 152; do
  SLATE_AMD_HB2ST_LDS=$kb timeout -k 10 200 python -u tools/probe/hb2st_time.py 16384 64 > gpurun_out/hb2st_lds$kb.log 2>&1 || { tail gpurun_out/hb2st_lds$kb.log; exit 1; }
  echo "lds=$kb KB: $(grep -h 'device\|phases' gpurun_out/hb2st_lds$kb.log | tr '\n' ' ')"
done
timeout -k 10 300 python -u tools/probe/tb2bd_time.py 8192 64
