#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_prof_csv.sh potrf2 --steps 1 --warmup 1 --check 0 || true
python3 tools/prof_csv_summary.py gpurun_out/pc_potrf2 12
python3 tools/prof_timeline.py gpurun_out/pc_potrf2 225
