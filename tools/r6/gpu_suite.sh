#!/bin/bash
# full GPU suite (round 6 end state)
set -o pipefail
mkdir -p gpurun_out/r6/suite
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r6/suite/gpu_suite.log 2>&1
rc=$?
tail -15 gpurun_out/r6/suite/gpu_suite.log
exit $rc
