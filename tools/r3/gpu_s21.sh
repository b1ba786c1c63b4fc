#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${TAG:-s21}; mkdir -p $D
timeout -k 10 200 python -u tools/probe/stedc_cprof.py > $D/stedc_cprof.log 2>&1 || { tail $D/stedc_cprof.log; exit 1; }
echo ok
