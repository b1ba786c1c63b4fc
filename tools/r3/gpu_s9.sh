#!/bin/bash
# heev phase spans (he2hb / hb2st / stedc / back-transforms)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${TAG:-s9}; mkdir -p $D
timeout -k 10 300 python -u tools/heev_phases.py 16384 256 > $D/heev_phases.log 2>&1 || { tail $D/heev_phases.log; exit 1; }
cat $D/heev_phases.log
