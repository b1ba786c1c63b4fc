"""One fp64 LU panel (ops.getrf, m x 512) after a warm-up: for rocprofv3 kernel traces."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from slate_amd import ops
m = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 512
A0 = torch.randn(m, nb, dtype=torch.float64).t().contiguous().t().cuda()
ipiv = torch.zeros(nb, dtype=torch.int64, device="cuda")
for _ in range(3):
    A = A0.clone(); ops.getrf(A, ipiv)
torch.cuda.synchronize()
print("done", m, nb)
