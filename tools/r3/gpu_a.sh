#!/bin/bash
# Round-3 first GPU pass: full GPU test suite, headline benches, RCCL 2-ranks-on-1-GPU probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3a
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3a/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/r3a/pytest_gpu.log
[ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && exit 1
timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r3a/bench_potrf.log 2>&1 || { echo potrf bench failed; tail gpurun_out/r3a/bench_potrf.log; exit 1; }
tail -1 gpurun_out/r3a/bench_potrf.log
timeout -k 10 200 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 > gpurun_out/r3a/bench_getrf.log 2>&1 || { echo getrf bench failed; tail gpurun_out/r3a/bench_getrf.log; exit 1; }
tail -1 gpurun_out/r3a/bench_getrf.log
timeout -k 10 200 python -u bench.py --routine geqrf --rows 65536 --size 8192 --nb 256 --steps 3 --warmup 1 > gpurun_out/r3a/bench_geqrf.log 2>&1 || { echo geqrf bench failed; tail gpurun_out/r3a/bench_geqrf.log; exit 1; }
tail -1 gpurun_out/r3a/bench_geqrf.log
timeout -k 10 200 python -u bench.py --routine gemm --steps 3 --warmup 1 > gpurun_out/r3a/bench_gemm.log 2>&1 || { echo gemm bench failed; tail gpurun_out/r3a/bench_gemm.log; exit 1; }
tail -1 gpurun_out/r3a/bench_gemm.log
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r3a/bench_potrf_hwq8.log 2>&1 || { echo potrf hwq8 failed; tail gpurun_out/r3a/bench_potrf_hwq8.log; exit 1; }
tail -1 gpurun_out/r3a/bench_potrf_hwq8.log
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 tools/probe/rccl_same_gpu.py > gpurun_out/r3a/rccl_probe.log 2>&1
echo "rccl probe rc=$?"; grep -v "^\[W\|amdgpu.ids" gpurun_out/r3a/rccl_probe.log | tail -8
