#!/bin/bash
# round 6 / a: advisor fixes (LU peer G > 1, parked update stream), the
# bench self-launch rehearsed with 2 gloo ranks sharing the GPU, 1-GPU bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6; mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_dist_gpu.py::test_lu_panel_peer_mailbox tests/test_nosync_gpu.py > $D/pytest_a.log 2>&1
rc=$?; tail -25 $D/pytest_a.log; [ $rc -eq 0 ] || exit $rc
SLATE_AMD_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --size 8192 --nb 512 --steps 2 --warmup 1 > $D/bench_selflaunch_2gloo.txt 2>&1
rc=$?; cat $D/bench_selflaunch_2gloo.txt | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > $D/bench_potrf_1gpu.txt 2>&1
rc=$?; cat $D/bench_potrf_1gpu.txt | tail -3; exit $rc
