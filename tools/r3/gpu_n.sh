#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && export PYTHONPATH="$GRAFT_REPO_ROOT"
O=gpurun_out/r3n
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_nosync_gpu.py -x -q --timeout 120 --timeout-method thread > $O/nosync.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/nosync.log
[ $rc -ne 0 ] && exit 1
HB2ST_PROBE_NOHOST=1 timeout -k 10 300 python -u tools/probe/hb2st_time.py 16384 64 > $O/hb2st_16384.log 2>&1
echo "rc=$?"; grep -v amdgpu.ids $O/hb2st_16384.log | tail -4
