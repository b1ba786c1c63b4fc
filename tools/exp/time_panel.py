"""Standalone timing of the LU panel (getrf_panel_ws) on one tall fp64 panel."""
import time, torch
from slate_amd import ops
for m, n in [(32768, 512), (16384, 512), (32768, 32)]:
    g = torch.Generator().manual_seed(1)
    A0 = torch.randn(m, n, dtype=torch.float64, generator=g).t().contiguous().t().cuda()
    ipiv = torch.zeros(n, dtype=torch.int64, device="cuda")
    for it in range(4):
        A = A0.clone()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ops.getrf(A, ipiv)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    print(f"panel {m}x{n}: {dt*1e3:.3f} ms  ({dt*1e6/n:.2f} us/column)", flush=True)
