#!/bin/bash
# heev phases (host spans + device spans), host vs device bulge chase,
# kernel stats of one heev (CSV)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pc_heev
timeout -k 10 300 python -u tools/heev_phases.py 16384 256 > gpurun_out/heev_phases_host.log 2>&1 || { cat gpurun_out/heev_phases_host.log; exit 1; }
cat gpurun_out/heev_phases_host.log
SLATE_AMD_HB2ST=device timeout -k 10 300 python -u tools/heev_phases.py 16384 256 > gpurun_out/heev_phases_dev.log 2>&1 || { cat gpurun_out/heev_phases_dev.log; exit 1; }
cat gpurun_out/heev_phases_dev.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pc_heev -o heev -- python3 tools/heev_phases.py 16384 256 > gpurun_out/pc_heev/run.log 2>&1
find gpurun_out/pc_heev -name "*kernel_trace.csv" -size +50M -delete
python3 tools/prof_csv_summary.py gpurun_out/pc_heev 20 || true
