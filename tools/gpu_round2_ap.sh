#!/bin/bash
# bench.py's multi-rank path on the GPU box: 2 and 4 ranks sharing cuda:0 over gloo
# (RCCL refuses two ranks on one GPU); checks the JSON line and info, not speed
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ranks
for np in 2 4; do
  for r in potrf getrf; do
    SLATE_AMD_DIST_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np \
      --master-addr 127.0.0.1 --master-port $((29600 + np)) bench.py --gpus $np --routine $r --size 8192 --nb 512 \
      --steps 1 --warmup 1 > gpurun_out/ranks/${r}_$np.log 2>&1 || { tail -20 gpurun_out/ranks/${r}_$np.log; exit 1; }
    echo "$r np=$np: $(grep -o '"grid": "[0-9x]*"\|"info_ok": [a-z]*\|"value": [0-9.]*' gpurun_out/ranks/${r}_$np.log | tr '\n' ' ')"
  done
done
