#!/bin/bash
# kernel trace of the native dgetrf bench (last step)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r5/u; mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/ng -o run -- ./slate_amd/bench_native getrf 32768 512 1 1 2 1 2 0 32768 > $D/ng.log 2>&1
echo "prof rc=$?"
