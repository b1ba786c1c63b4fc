#!/bin/bash
# Round-2: TSQR on the GPU (multi-rank rehearsal) + QR GPU tests + geqrf bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py tests/test_qr.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_qr_gpu.log 2>&1
rc=$?; echo "qr/dist gpu tests rc=$rc"; tail -4 gpurun_out/pytest_qr_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u bench.py --routine geqrf --m 65536 --n 8192 --nb 256 --steps 3 --warmup 1 > gpurun_out/bench_geqrf.log 2>&1 || exit 1
tail -1 gpurun_out/bench_geqrf.log
