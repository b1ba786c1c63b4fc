#!/bin/bash
# graph potrf timing (kernel-node zeroing), then a dpotrf sweep: group size x lookahead
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && export PYTHONPATH="$GRAFT_REPO_ROOT"
O=gpurun_out/r3j
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_nosync_gpu.py -x -q --timeout 120 --timeout-method thread > $O/nosync.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/nosync.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 200 python -u tools/probe/graph_time.py > $O/graph_time.log 2>&1
echo "graph_time rc=$?"; grep -v amdgpu.ids $O/graph_time.log | tail -6
for g in 2 3 4; do for la in 1 2; do
  SLATE_AMD_POTRF_GROUP=$g timeout -k 10 150 python -u bench.py --steps 4 --warmup 2 --lookahead $la > $O/potrf_g${g}_la${la}.log 2>&1 || { echo "potrf g=$g la=$la failed"; tail -3 $O/potrf_g${g}_la${la}.log; exit 1; }
  echo "g=$g la=$la $(tail -1 $O/potrf_g${g}_la${la}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
