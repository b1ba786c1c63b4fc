"""GEMM efficiency vs k for the potrf trailing-update shape (N,T), ours vs hipBLASLt (torch, calibration)."""
import sys, time, torch
sys.path.insert(0, '.')
from tools.bench_gemm import run

for k in (256, 512, 1024, 2048):
    run('d', 'N', 'T', 24576, 24576, k, reps=3)
    run('d', 'N', 'N', 24576, 24576, k, reps=3)
for k in (512, 1024):
    a = torch.randn(24576, k, dtype=torch.float64, device='cuda'); c = torch.randn(24576, 24576, dtype=torch.float64, device='cuda')
    torch.addmm(c, a, a.t(), beta=1.0, alpha=-1.0, out=c); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3): torch.addmm(c, a, a.t(), beta=1.0, alpha=-1.0, out=c)
    torch.cuda.synchronize(); dt = (time.perf_counter() - t0) / 3
    print(f"hipBLASLt (torch) NT 24576x24576x{k}: {dt*1e3:.3f} ms {2*24576*24576*k/dt/1e12:.2f} TF/s", flush=True)
run('d', 'N', 'T', 16384, 16384, 16384, reps=2)
