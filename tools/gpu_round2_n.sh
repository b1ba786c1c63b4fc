#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_eig_svd.py -x -v --timeout 150 --timeout-method thread -m gpu > gpurun_out/pytest_eig.log 2>&1 || { tail -40 gpurun_out/pytest_eig.log; exit 1; }
tail -2 gpurun_out/pytest_eig.log
for band in 64 32; do
  SLATE_AMD_HB2ST=device timeout -k 10 300 python -u tools/heev_phases.py 16384 256 $band > gpurun_out/heev_phases_$band.log 2>&1 || { cat gpurun_out/heev_phases_$band.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/heev_phases_$band.log | grep -v "  host"
done
