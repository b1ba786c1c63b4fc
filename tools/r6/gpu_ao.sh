#!/bin/bash
# Python heev: Q1 group merges on the panel stream during the chase (on / off)
set -o pipefail
mkdir -p gpurun_out/r6/ao
timeout -k 10 400 python -u -m pytest tests/test_eig_svd.py tests/test_kernel_census_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r6/ao/tests.log 2>&1 || { tail -30 gpurun_out/r6/ao/tests.log; exit 1; }
tail -2 gpurun_out/r6/ao/tests.log
timeout -k 10 300 python bench.py --routine heev --size 16384 --nb 256 --steps 3 --warmup 1 > gpurun_out/r6/ao/heev_on.json 2> gpurun_out/r6/ao/heev_on.err || { tail -5 gpurun_out/r6/ao/heev_on.err; exit 1; }
cat gpurun_out/r6/ao/heev_on.json
SLATE_AMD_HEEV_OVERLAP=0 timeout -k 10 300 python bench.py --routine heev --size 16384 --nb 256 --steps 3 --warmup 1 > gpurun_out/r6/ao/heev_off.json 2> gpurun_out/r6/ao/heev_off.err || { tail -5 gpurun_out/r6/ao/heev_off.err; exit 1; }
cat gpurun_out/r6/ao/heev_off.json
