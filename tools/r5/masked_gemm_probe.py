"""The 2x4 dpotrf trailing update of rank (0, 0), step 0, in isolation:
C(15872 x 7168) -= P(15872 x 512) L(7168 x 512)^T with the block-cyclic
lower mask, against the same GEMM unmasked and a dense square of equal flops."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from slate_amd import ops

dev = torch.device("cuda", 0)
cm = lambda m, n: torch.randn(n, m, dtype=torch.float64, device=dev).t()   # noqa: E731
buf = cm(16384, 8192)
P = cm(15872, 512)
L = cm(7680, 512)
C = buf[512:, 1024:]
Lc = L[512:]
mask = (1, 512, 2, 0, 4, 0, 512, 1024, 0)


def t(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


fl_full = 2.0 * 15872 * 7168 * 512
for name, fn, fl in [
    ("masked (kept 48%)", lambda: ops.gemm(-1.0, P, Lc, 1.0, C, 'N', 'T', mask), fl_full * 0.4839),
    ("unmasked", lambda: ops.gemm(-1.0, P, Lc, 1.0, C, 'N', 'T'), fl_full),
    ("mask keeping all", lambda: ops.gemm(-1.0, P, Lc, 1.0, C, 'N', 'T', (1, 512, 2, 0, 4, 0, 512, 1024, 1 << 40)), fl_full),
    ("mask skipping all", lambda: ops.gemm(-1.0, P, Lc, 1.0, C, 'N', 'T', (1, 512, 2, 0, 4, 0, 512, 1024, -(1 << 40))), 1.0),
    ("kept-size rectangle", lambda: ops.gemm(-1.0, P[:7424], Lc, 1.0, C[:7424], 'N', 'T'), fl_full * 7424 / 15872),
    ("unmasked, C contiguous ld", lambda: ops.gemm(-1.0, P, Lc, 1.0, cm(15872, 7168), 'N', 'T'), fl_full),
]:
    ms = t(fn)
    print(f"{name:28s} {ms * 1e3:9.1f} us  {fl / ms / 1e9:6.1f} TF/s", flush=True)
print("strides: C", C.stride(), "P", P.stride(), "Lc", Lc.stride(), "ptr mod 16", C.data_ptr() % 16, P.data_ptr() % 16, Lc.data_ptr() % 16)
