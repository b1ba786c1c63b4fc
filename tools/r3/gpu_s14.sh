#!/bin/bash
# hb2st memory mode / threads sweep with early publication
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${TAG:-s14}; mkdir -p $D
for cfg in "SLATE_AMD_HB2ST_MEM=uncached" "SLATE_AMD_HB2ST_MEM=finegrained" "SLATE_AMD_HB2ST_MEM=cached" "SLATE_AMD_HB2ST_THREADS=512" "SLATE_AMD_HB2ST_EARLY=0"; do
  env $cfg HB2ST_PROBE_NOHOST=1 timeout -k 10 120 python -u tools/probe/hb2st_time.py 16384 64 > $D/hb2st.log 2>&1 || { echo "$cfg failed"; tail -3 $D/hb2st.log; exit 1; }
  echo "$cfg: $(grep device $D/hb2st.log) | $(grep phases $D/hb2st.log | cut -c1-90)"
done
