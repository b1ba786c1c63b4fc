#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6/s
PYTHONPATH=$PWD:$PWD/tests timeout -k 10 300 python -u tools/r6/census_stack.py > gpurun_out/r6/s/stack.log 2>&1
rc=$?
tail -60 gpurun_out/r6/s/stack.log
exit $rc
