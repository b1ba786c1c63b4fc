#!/bin/bash
# every tester routine on the GPU (device target), plus norm/eig GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/tester_all.py --dim 300 --nb 64 --type d,z > gpurun_out/tester_all.log 2>&1; rc=$?
grep -h "FAILED" gpurun_out/tester_all.log | head -40
exit $rc
