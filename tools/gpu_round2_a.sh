#!/bin/bash
# Round-2 first GPU pass: kernel/driver tests, 1-GPU bench, RCCL 2-ranks-on-1-GPU probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench1.log 2>&1 || { echo bench failed; tail gpurun_out/bench1.log; exit 1; }
cat gpurun_out/bench1.log | tail -2
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 tools/probe/rccl_same_gpu.py > gpurun_out/rccl_probe.log 2>&1
echo "rccl probe rc=$?"; tail -5 gpurun_out/rccl_probe.log
