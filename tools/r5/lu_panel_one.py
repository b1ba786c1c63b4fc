"""One m x 512 fp64 LU panel (ops.getrf) repeated, for counter runs."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from slate_amd import ops
m = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
g = torch.Generator().manual_seed(1)
A0 = torch.randn(m, 512, dtype=torch.float64, generator=g).t().contiguous().t().cuda()
ipiv = torch.zeros(512, dtype=torch.int64, device="cuda")
for it in range(4):
    A = A0.clone()
    ops.getrf(A, ipiv)
torch.cuda.synchronize()
print("done", m)
