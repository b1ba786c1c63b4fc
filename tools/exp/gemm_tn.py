"""W = V^T C for the QR trailing update shapes: our MFMA GEMM vs torch (rocBLAS/hipBLASLt)."""
import time, torch
from slate_amd import ops
def t(fn, reps=5):
    fn(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps): fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps
for m, n in [(65536, 7936), (65536, 4096), (57600, 256), (61440, 2048)]:
    V = torch.randn(256, m, dtype=torch.float64, device="cuda").t()      # m x 256 col-major
    C = torch.randn(n, m, dtype=torch.float64, device="cuda").t()        # m x n col-major
    W = ops.colmajor_empty(256, n, torch.float64, V.device)
    a = t(lambda: ops.gemm(1.0, V, C, 0.0, W, transA='T'))
    b = t(lambda: torch.matmul(V.t(), C))
    fl = 2 * 256 * m * n
    print(f"TN m={m} n={n}: ours {a*1e6:.0f} us {fl/a/1e12:.1f} TF/s   torch {b*1e6:.0f} us {fl/b/1e12:.1f} TF/s", flush=True)
    W2 = ops.colmajor_empty(256, n, torch.float64, V.device)
    c = t(lambda: ops.gemm(-1.0, V, W2, 1.0, C))
    print(f"NN m={m} n={n} k=256: ours {c*1e6:.0f} us {fl/c/1e12:.1f} TF/s", flush=True)
