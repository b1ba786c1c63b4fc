"""Latency of the fp64 tile Cholesky (the diagonal tile of the distributed
potrf, n = 512 by default), variant 0 = one-CU potrf_lds, 1 = multi-workgroup
potrf_mc, alone and next to a concurrent trailing-update GEMM on another
stream (the panel stream's priority).  One line per variant."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from slate_amd import ops, _native

dev = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
H = _native.hip()
g = torch.Generator(device=dev).manual_seed(1)
X = torch.rand(n, n, dtype=torch.float64, device=dev, generator=g)
S = (X @ X.T + n * torch.eye(n, dtype=torch.float64, device=dev)).T.contiguous().T
A = S.clone()
info = torch.zeros(1, dtype=torch.int64, device=dev)
M = 16384
Ga = ops.colmajor_zeros(M, 512, torch.float64, dev)
Gc = ops.colmajor_zeros(M, M, torch.float64, dev)
side = torch.cuda.Stream(device=dev)
hi = torch.cuda.Stream(device=dev, priority=-1)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def run(v, st):
    H.potrf_tile_variant(v, n, A.data_ptr(), A.stride(1), info.data_ptr(), st.cuda_stream)


for v in (0, 1):
    cur = torch.cuda.current_stream()
    for _ in range(5):
        A.copy_(S)
        run(v, cur)
    torch.cuda.synchronize()
    ts = []
    for _ in range(20):
        A.copy_(S)
        e0.record()
        run(v, cur)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    L = torch.tril(A)
    res = float((L @ L.T - S).norm() / S.norm())
    tl = []
    for _ in range(10):
        A.copy_(S)
        torch.cuda.synchronize()
        with torch.cuda.stream(side):
            ops.gemm(-1.0, Ga, Ga, 1.0, Gc, 'N', 'T')
        with torch.cuda.stream(hi):
            e0.record()
            run(v, hi)
            e1.record()
        torch.cuda.synchronize()
        tl.append(e0.elapsed_time(e1) * 1e3)
    print(f"n={n} variant={['potrf_lds', 'potrf_mc'][v]} alone_us min/med={min(ts):.1f}/{sorted(ts)[len(ts)//2]:.1f} "
          f"loaded_us med={sorted(tl)[len(tl)//2]:.1f} info={int(info)} res={res:.2e}", flush=True)
