"""Latency of the tile potrf (n = 512 diagonal tile of the distributed
Cholesky) for the diagonal block size in SLATE_AMD_POTRF_DIAG, alone and
under a concurrent trailing-update GEMM load.  One line per run."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from slate_amd import ops

dev = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
g = torch.Generator(device=dev).manual_seed(1)
X = torch.rand(n, n, dtype=torch.float64, device=dev, generator=g)
S = (X @ X.T + n * torch.eye(n, dtype=torch.float64, device=dev)).T.contiguous().T
A = S.clone()
info = torch.zeros(1, dtype=torch.int64, device=dev)
for _ in range(5):
    A.copy_(S); ops.potrf('L', A, info)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ts = []
for _ in range(20):
    A.copy_(S)
    e0.record(); ops.potrf('L', A, info); e1.record(); torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) * 1e3)
L = torch.tril(A)
res = float((L @ L.T - S).norm() / S.norm())
# under load: a big GEMM on another stream
M = 16384
Ga = ops.colmajor_zeros(M, 512, torch.float64, dev); Gc = ops.colmajor_zeros(M, M, torch.float64, dev)
side = torch.cuda.Stream(device=dev)
hi = torch.cuda.Stream(device=dev, priority=-1)     # the panel stream's priority
tl = []
for _ in range(10):
    A.copy_(S); torch.cuda.synchronize()
    with torch.cuda.stream(side):
        ops.gemm(-1.0, Ga, Ga, 1.0, Gc, 'N', 'T')
    with torch.cuda.stream(hi):
        e0.record(); ops.potrf('L', A, info); e1.record()
    torch.cuda.synchronize()
    tl.append(e0.elapsed_time(e1) * 1e3)
print(f"n={n} diag={os.environ.get('SLATE_AMD_POTRF_DIAG', '512')} alone_us={min(ts):.1f}/{sorted(ts)[len(ts)//2]:.1f} "
      f"loaded_us={sorted(tl)[len(tl)//2]:.1f} info={int(info)} res={res:.2e}", flush=True)
