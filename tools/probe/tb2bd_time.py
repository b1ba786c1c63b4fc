"""Time of the GPU bidiagonal chase (hb2st.hip tb2bd_kernel) vs the host
pipeline for a random upper band; argv: n b."""
import os
import sys
import time
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from slate_amd.models import svd as S

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
b = int(sys.argv[2]) if len(sys.argv) > 2 else 64
g = torch.Generator().manual_seed(1)
X = torch.randn(n, n, generator=g, dtype=torch.float64)
i = torch.arange(n)
dl = i[None, :] - i[:, None]
B = torch.where((dl >= 0) & (dl <= b), X, torch.zeros_like(X))
Bd = B.cuda()
S.tb2bd(Bd, b)
torch.cuda.synchronize()
t0 = time.perf_counter()
d, e, F = S.tb2bd(Bd, b)
torch.cuda.synchronize()
print(f"device tb2bd n={n} b={b}: {time.perf_counter() - t0:.3f} s", flush=True)
t0 = time.perf_counter()
d2, e2, F2 = S.tb2bd(B, b)
print(f"host   tb2bd n={n} b={b}: {time.perf_counter() - t0:.3f} s", flush=True)
s1 = torch.linalg.svdvals(torch.diag(d) + torch.diag(e, 1))
s2 = torch.linalg.svdvals(torch.diag(d2) + torch.diag(e2, 1))
print("sv diff", float((s1 - s2).abs().max()), flush=True)
