#!/bin/bash
# wave-per-root secular/zhat kernels: eig GPU tests, device gelqf test, heev phases (wave vs thread)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_eig_svd.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "stedc or heev or svd or hegv or gelqf or tb2bd or hb2st" > gpurun_out/pytest_al.log 2>&1 || { tail -30 gpurun_out/pytest_al.log; exit 1; }
tail -1 gpurun_out/pytest_al.log
for w in 1 0; do
  SLATE_AMD_SECULAR_WAVE=$w timeout -k 10 300 python -u tools/heev_phases.py 16384 256 > gpurun_out/heev_phases_w$w.log 2>&1 || { tail gpurun_out/heev_phases_w$w.log; exit 1; }
  echo "wave=$w: $(grep -h 'heev n=\|device   stedc' gpurun_out/heev_phases_w$w.log | tr '\n' ' ')"
done
