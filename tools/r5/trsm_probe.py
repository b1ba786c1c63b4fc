"""Panel solve X L^T = B (dpotrf's trsm, B: m x n, L: n x n lower) alone on
MI355X: the current kernel path vs SLATE_AMD_TRSM_RLT_REC=1 (run twice);
python tools/r5/trsm_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from slate_amd import ops

dev = torch.device("cuda", 0)
cm = lambda m, n: torch.randn(n, m, dtype=torch.float64, device=dev).t()   # noqa: E731
n = 512
Lf = torch.randn(n, n, dtype=torch.float64, device=dev)
S = Lf @ Lf.T + n * torch.eye(n, dtype=torch.float64, device=dev)
L = torch.linalg.cholesky(S).T.contiguous().T        # column-major lower
for m in (4096, 8192, 16384, 32256):
    B0 = cm(m, n)
    B = B0.clone()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ops.trsm('R', 'L', 'T', 'N', 1.0, L, B)
    torch.cuda.synchronize()
    X = B.clone()
    err = ((X @ L.T - B0).abs().max() / B0.abs().max()).item()
    reps = 10
    e0.record()
    for _ in range(reps):
        B.copy_(B0)
        ops.trsm('R', 'L', 'T', 'N', 1.0, L, B)
    e1.record()
    torch.cuda.synchronize()
    e2, e3 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e2.record()
    for _ in range(reps):
        B.copy_(B0)
    e3.record()
    torch.cuda.synchronize()
    ms = (e0.elapsed_time(e1) - e2.elapsed_time(e3)) / reps
    print(f"rec={os.environ.get('SLATE_AMD_TRSM_RLT_REC', '0')} m={m:6d} n={n}: {ms * 1e3:7.1f} us "
          f"{m * n * n / ms / 1e9:6.1f} TF/s  err {err:.1e}", flush=True)
