#!/bin/bash
# LU panel: tagged vs counter base case timing, LU tests, dgetrf bench + profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${TAG:-lu2}; mkdir -p $D
NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=COLL timeout -k 10 120 python -u tools/probe/nccl_stream_probe.py > $D/nccl_probe.log 2>&1; grep -E "side stream|opCount" $D/nccl_probe.log | tail -8

timeout -k 10 120 python -u tools/probe/lu_panel_time.py > $D/panel_tag.log 2>&1 || { tail $D/panel_tag.log; exit 1; }
cat $D/panel_tag.log | grep -v amdgpu.ids
SLATE_AMD_LU_PANEL=counter timeout -k 10 120 python -u tools/probe/lu_panel_time.py > $D/panel_cnt.log 2>&1 || { tail $D/panel_cnt.log; exit 1; }
cat $D/panel_cnt.log | grep -v amdgpu.ids
timeout -k 10 300 python -u -m pytest tests/test_lu_rowmajor_gpu.py tests/test_nosync_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "lu or getrf or laswp or nosync or graph or census" > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/pytest.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 200 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 > $D/bench_getrf.log 2>&1 || { tail $D/bench_getrf.log; exit 1; }
tail -1 $D/bench_getrf.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run -- python3 -u bench.py --routine getrf --lookahead 2 --steps 1 --warmup 1 > $D/prof.log 2>&1 || { tail -5 $D/prof.log; exit 1; }
echo prof ok
timeout -k 10 300 python -u tools/check_dist_gpu.py 4 > $D/dist4.log 2>&1 || { tail -20 $D/dist4.log; exit 1; }
tail -8 $D/dist4.log
