"""Run the multi-workgroup tile Cholesky (potrf_mc) N times alone, for a
rocprofv3 kernel trace (per-launch durations of the P / U kernels)."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from slate_amd import _native

dev = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
H = _native.hip()
g = torch.Generator(device=dev).manual_seed(1)
X = torch.rand(n, n, dtype=torch.float64, device=dev, generator=g)
S = (X @ X.T + n * torch.eye(n, dtype=torch.float64, device=dev)).T.contiguous().T
A = S.clone()
info = torch.zeros(1, dtype=torch.int64, device=dev)
st = torch.cuda.current_stream().cuda_stream
for _ in range(reps):
    A.copy_(S)
    H.potrf_tile_variant(1, n, A.data_ptr(), A.stride(1), info.data_ptr(), st)
torch.cuda.synchronize()
print("done", int(info))
