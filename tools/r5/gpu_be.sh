#!/bin/bash
# rocprofv3 kernel stats: 1-GPU dpotrf bench and the 2x4 loopback rank 0 (link 10/150)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r5/be; mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/bench -o run -- python3 bench.py --steps 2 --warmup 1 > $D/bench.log 2>&1
echo "bench prof rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/lb -o run -- python3 tools/r5/loopback_critpath.py --grid 2x4 --ranks 0 --steps 1 --link 10,150 > $D/lb.log 2>&1
echo "lb prof rc=$?"
