#!/bin/bash
# native p x q QR checks first, then the full GPU suite + smoke + benches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5/i; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_native_gpu.py -x -v --timeout 240 --timeout-method thread > $D/native.log 2>&1
rc=$?; grep -E "PASS|FAIL|check (geqrf|gels)" $D/native.log | head -60
[ $rc -ne 0 ] && { grep -E "Error|assert" $D/native.log | head -20; exit 1; }
TAG=i bash tools/r5/gpu_full.sh
