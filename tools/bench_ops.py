"""Isolated timings of the potrf-path device ops (one process, interleaved)."""
import os, sys, time, torch
sys.path.insert(0, '.')
from slate_amd import ops

def cm(m, n, dt=torch.float64):
    return torch.randn(n, m, dtype=dt, device='cuda').t()

def timeit(fn, reps=10):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us

def spd(n):
    X = torch.randn(n, n, dtype=torch.float64, device='cuda')
    S = X @ X.T + n * torch.eye(n, dtype=torch.float64, device='cuda')
    return S

for n in (128, 512):
    S = spd(n)
    A = cm(n, n); 
    def f():
        A.copy_(S); ops.potrf('L', A)
    print(f"potrf tile n={n}: {timeit(f):.1f} us", flush=True)
L = torch.tril(spd(512)); L.diagonal().add_(100.0)
Lc = cm(512, 512); Lc.copy_(L)
for m in (4096, 32768):
    B = cm(m, 512)
    print(f"trsm R L C N m={m} n=512: {timeit(lambda: ops.trsm('R','L','T','N',1.0,Lc,B)):.1f} us", flush=True)
for m in (4096, 32768):
    P = cm(m, 512); C = cm(m, m)
    mask = (1, 1 << 40, 1, 0, 1, 0, 0, 0, 0)
    t = timeit(lambda: ops.gemm(-1.0, P, P, 1.0, C, 'N', 'T', mask), reps=3)
    print(f"masked syrk m={m} k=512: {t:.1f} us  {m*m*512/t/1e6:.1f} TF/s", flush=True)
    t = timeit(lambda: ops.gemm(-1.0, P, P, 1.0, C, 'N', 'T'), reps=3)
    print(f"full gemm m={m} k=512: {t:.1f} us  {2*m*m*512/t/1e6:.1f} TF/s", flush=True)
