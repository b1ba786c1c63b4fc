"""Masked (lower) fp64 trailing-update GEMM: compact lower-triangle launch
(SLATE_AMD_GEMM_TRI=1, default) vs the full grid with early-exit blocks
(SLATE_AMD_GEMM_TRI=0).  Shapes of the n = 32768, nb = 512 potrf updates."""
import os
import sys
import time
sys.path.insert(0, '.')
import torch  # noqa: E402
from slate_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
for m in (32768 - 1024, 24576, 16384, 8192, 4096):
    n, k = m - 1024, 512
    A = torch.randn(k, m, device=dev, dtype=torch.float64).mT
    C = torch.randn(n + 1024, m, device=dev, dtype=torch.float64).mT[:, :n]
    mask = (1, 1 << 40, 1, 0, 1, 0, 0, 1024, 0)
    flops = 2.0 * k * (m * n - n * n / 2)
    for tri in ("1", "0", "1", "0"):
        os.environ["SLATE_AMD_GEMM_TRI"] = tri
        for _ in range(2):
            ops.gemm(-1.0, A, A[1024:], 1.0, C, 'N', 'T', mask)
        torch.cuda.synchronize()
        reps = 10
        t0 = time.perf_counter()
        for _ in range(reps):
            ops.gemm(-1.0, A, A[1024:], 1.0, C, 'N', 'T', mask)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        print(f"m={m} n={n} k={k} tri={tri}: {dt * 1e3:.3f} ms  {flops / dt / 1e12:.1f} TF/s", flush=True)
