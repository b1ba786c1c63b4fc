"""Debug: persistent LU base case vs torch on small shapes."""
import torch
from slate_amd import ops

def cm(m, n, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, m, dtype=torch.float64, generator=g).t().contiguous().t().cuda() if False else \
        torch.randn(m, n, dtype=torch.float64, generator=g).t().contiguous().t().cuda()

for m, n in [(1000, 1), (1000, 2), (1000, 8), (1000, 32), (600, 32), (1000, 64), (1000, 96), (2048, 32)]:
    A0 = cm(m, n, 31)
    A = A0.clone()
    ipiv = torch.zeros(n, dtype=torch.int64, device="cuda")
    info = ops.getrf(A, ipiv)
    torch.cuda.synchronize()
    LU_ref, piv_ref = torch.linalg.lu_factor(A0.cpu())
    pr = (piv_ref[:n].to(torch.int64) - 1)
    ip = ipiv.cpu()
    bad = (ip != pr).nonzero().flatten().tolist()
    err = ((A.cpu() - LU_ref).abs().max() / A0.abs().max()).item()
    print(f"m={m} n={n} info={int(info.item())} first bad pivots={bad[:5]} ipiv={ip[:6].tolist()} ref={pr[:6].tolist()} err={err:.2e}", flush=True)
