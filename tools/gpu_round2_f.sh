#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/probe/heev_breakdown.py 8192 256 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 400 python -u bench.py --routine heev --n 16384 --nb 256 --steps 1 --warmup 0 2>&1 | grep -v amdgpu.ids | tail -2 || exit 1
