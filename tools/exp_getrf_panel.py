"""Panel LU micro-benchmark: base block (32 cols) and full nb=512 panels."""
import sys, time, torch
sys.path.insert(0, '.')
from slate_amd import ops

dev = torch.device('cuda')
for m, n in [(32768, 32), (8192, 32), (32768, 512), (4096, 512)]:
    A0 = torch.randn(n, m, dtype=torch.float64, device=dev).t()
    A = A0.clone().t().contiguous().t() if False else torch.empty_like(A0)
    piv = torch.zeros(n, dtype=torch.int64, device=dev)
    info = torch.zeros(1, dtype=torch.int64, device=dev)
    for it in range(3):
        A.copy_(A0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ops.getrf(A, piv, info)
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
    print(f"panel getrf {m}x{n}: {t*1e3:.3f} ms", flush=True)
