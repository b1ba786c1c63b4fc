"""Locate the hipGraph capture failure step by step: capture one op at a time
on a side stream (torch.cuda.CUDAGraph), replay, compare with an eager run.
faulthandler prints the Python stack if the process segfaults."""
import faulthandler
import sys

import torch

faulthandler.enable()
import slate_amd as sl  # noqa: E402
from slate_amd import ops  # noqa: E402

dev = torch.device("cuda")


def step(name, fn, check):
    print(f"== {name}: warm-up", flush=True)
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    print(f"== {name}: capture", flush=True)
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s, capture_error_mode="relaxed"):
            fn()
    torch.cuda.synchronize()
    print(f"== {name}: replay", flush=True)
    g.replay()
    torch.cuda.synchronize()
    print(f"== {name}: {check()}", flush=True)


n = 1024
A = ops.colmajor_empty(n, n, torch.float64, dev)
A.copy_(torch.randn(n, n, dtype=torch.float64, device=dev))
B = ops.colmajor_empty(n, n, torch.float64, dev)
B.copy_(torch.randn(n, n, dtype=torch.float64, device=dev))
C = ops.colmajor_zeros(n, n, torch.float64, dev)
step("gemm", lambda: ops.gemm(1.0, A, B, 0.0, C), lambda: float((C - A @ B).abs().max()))

S0 = A @ A.T + n * torch.eye(n, dtype=torch.float64, device=dev)
T = ops.colmajor_empty(512, 512, torch.float64, dev)
info = torch.zeros(1, dtype=torch.int64, device=dev)


def tile():
    T.copy_(S0[:512, :512])
    ops.potrf('L', T, info)


step("potrf_tile", tile, lambda: float((torch.tril(T) @ torch.tril(T).T - S0[:512, :512]).abs().max()))

X = ops.colmajor_empty(n, 64, torch.float64, dev)


def trsm():
    X.copy_(B[:, :64])
    ops.trsm('L', 'L', 'N', 'N', 1.0, S0, X)


step("trsm", trsm, lambda: float((torch.tril(S0) @ X - B[:, :64]).abs().max()))

which = sys.argv[1] if len(sys.argv) > 1 else "all"
if which in ("all", "potrf"):
    N = 4096
    H = sl.HermitianMatrix(sl.Uplo.Lower, N, nb=512, device=dev)
    H.insertLocalTiles(device=dev)
    sl.generate_matrix(H, "poev", seed=3)
    buf = H.storage.local[H.storage.origin_slot]
    H0 = buf[:N, :N].clone()

    def chk():
        L = torch.tril(buf[:N, :N])
        S = torch.tril(H0) + torch.tril(H0, -1).mT
        return float((L @ L.mT - S).norm() / S.norm())

    print("== potrf Option.UseGraph: first call (capture + replay)", flush=True)
    info = sl.potrf(H, {sl.Option.Lookahead: 1, sl.Option.UseGraph: True})
    torch.cuda.synchronize()
    print("== potrf graph info", info, "err", chk(), flush=True)
    for it in range(3):
        buf[:N, :N].copy_(H0)
        info = sl.potrf(H, {sl.Option.Lookahead: 1, sl.Option.UseGraph: True})
        torch.cuda.synchronize()
        print("== potrf graph replay", it, "info", info, "err", chk(), flush=True)
print("probe done", flush=True)
