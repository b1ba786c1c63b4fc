"""Experiment: CU-masked streams for the panel chain vs the trailing GEMM.

1. placement probe: which XCC / CU ids blocks land on (default stream and a
   stream masked to the first k CU-mask bits);
2. panel chain (potrf_tile 512 + trsm m x 512) concurrently with a big
   trailing GEMM, for several mask splits.
"""
import sys
import time
from collections import Counter

import torch

sys.path.insert(0, '.')
from slate_amd import _native, ops  # noqa: E402

dev = torch.device('cuda')
H = _native.hip()
ncu = H.cu_count(0)
print("CUs", ncu, flush=True)


def probe(st_handle, nblk=4096):
    out = torch.zeros(2 * nblk, dtype=torch.int32, device=dev)
    H.placement_probe(out.data_ptr(), nblk, st_handle)
    torch.cuda.synchronize()
    v = out.view(-1, 2).cpu().tolist()
    xcc = Counter(int(x[1]) & 0xf for x in v)
    cus = Counter(((int(x[1]) & 0xf), (int(x[0]) >> 8) & 0xf, (int(x[0]) >> 13) & 0x3, (int(x[0]) >> 12) & 1)
                  for x in v)
    return xcc, len(cus)


def mask_words(bits):
    w = [0] * ((ncu + 31) // 32)
    for b in bits:
        w[b // 32] |= 1 << (b % 32)
    return w


cur = torch.cuda.current_stream().cuda_stream
print("default:", probe(cur), flush=True)
for k in (8, 16, 32):
    h = H.stream_create_cu_mask(0, mask_words(range(k)))
    print(f"first {k} bits:", probe(h), flush=True)
    h2 = H.stream_create_cu_mask(0, mask_words(range(0, ncu, ncu // k)))
    print(f"strided {k} bits:", probe(h2), flush=True)

# ---------------------------------------------------------------- timing
n, nb = 32768, 512
m = n - nb
torch.manual_seed(0)
C = ops.colmajor_empty(n, n, torch.float64, dev)
C.normal_()
Lp = ops.colmajor_empty(m, nb, torch.float64, dev)
Lp.normal_()
S = torch.randn(nb, nb, dtype=torch.float64, device=dev)
S = (S @ S.T + nb * torch.eye(nb, dtype=torch.float64, device=dev)).t().contiguous().t()
Pm = ops.colmajor_empty(m, nb, torch.float64, dev)
Pm.normal_()
info = torch.zeros(1, dtype=torch.int64, device=dev)


def chain(reps=8):
    for _ in range(reps):
        T = S.clone()
        ops.potrf('L', T, info)
        ops.trsm('R', 'L', 'T', 'N', 1.0, T, Pm)


def trailing():
    ops.gemm(-1.0, Lp[:16384], Lp[:16384], 1.0, C[:16384, :16384], transB='T')


def timeit(fn, st):
    torch.cuda.synchronize()
    with torch.cuda.stream(st):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
    return e0, e1


def run(name, ps, us):
    # warm
    with torch.cuda.stream(ps):
        chain(1)
    with torch.cuda.stream(us):
        trailing()
    torch.cuda.synchronize()
    # alone
    a0, a1 = timeit(chain, ps)
    torch.cuda.synchronize()
    b0, b1 = timeit(lambda: [trailing() for _ in range(6)], us)
    torch.cuda.synchronize()
    t_chain = a0.elapsed_time(a1)
    t_tr = b0.elapsed_time(b1)
    # concurrent
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    b0, b1 = timeit(lambda: [trailing() for _ in range(6)], us)
    a0, a1 = timeit(chain, ps)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    print(f"{name:28s} chain alone {t_chain:7.2f} ms  gemm alone {t_tr:7.2f} ms | "
          f"concurrent chain {a0.elapsed_time(a1):7.2f} gemm {b0.elapsed_time(b1):7.2f} wall {wall:7.2f}",
          flush=True)


hi = torch.cuda.Stream(priority=-1)
lo = torch.cuda.Stream(priority=0)
run("default hi/lo", hi, lo)
for k in (8, 16, 32):
    for layout in ("first", "strided"):
        bits = list(range(k)) if layout == "first" else list(range(0, ncu, ncu // k))
        rest = [b for b in range(ncu) if b not in set(bits)]
        ph = torch.cuda.ExternalStream(H.stream_create_cu_mask(0, mask_words(bits)))
        uh = torch.cuda.ExternalStream(H.stream_create_cu_mask(0, mask_words(rest)))
        run(f"{layout} {k}: panel|rest", ph, uh)
        run(f"{layout} {k}: panel=all|rest", hi, uh)
