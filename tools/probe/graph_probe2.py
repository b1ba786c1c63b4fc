"""Which part of the multi-stream potrf capture fails: (A) torch fork/join
over two plain streams, (B) over the slate_amd pipeline streams,
(C) the potrf driver with SLATE_AMD_SERIAL=1 (one stream).  argv[1] picks."""
import faulthandler
import os
import sys

import torch

faulthandler.enable()
which = sys.argv[1]
if len(sys.argv) > 2:
    os.environ["SLATE_AMD_DEBUG_POTRF_SKIP"] = sys.argv[2]
import slate_amd as sl  # noqa: E402
from slate_amd import ops  # noqa: E402
from slate_amd.parallel.streams import StreamSet  # noqa: E402

dev = torch.device("cuda")
n = 1024
A = ops.colmajor_empty(n, n, torch.float64, dev)
A.copy_(torch.randn(n, n, dtype=torch.float64, device=dev))
C1 = ops.colmajor_zeros(n, n, torch.float64, dev)
C2 = ops.colmajor_zeros(n, n, torch.float64, dev)


def forkjoin(s1, s2):
    cur = torch.cuda.current_stream()
    ev = torch.cuda.Event()
    ev.record(cur)
    s1.wait_event(ev)
    s2.wait_event(ev)
    with torch.cuda.stream(s1):
        ops.gemm(1.0, A, A, 0.0, C1)
    e1 = torch.cuda.Event()
    e1.record(s1)
    with torch.cuda.stream(s2):
        s2.wait_event(e1)
        ops.gemm(1.0, C1, A, 0.0, C2)
    e2 = torch.cuda.Event()
    e2.record(s2)
    e3 = torch.cuda.Event()
    e3.record(s1)
    cur.wait_event(e2)
    cur.wait_event(e3)


def cap(fn):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    cs = torch.cuda.Stream()
    cs.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cs):
        with torch.cuda.graph(g, stream=cs, capture_error_mode="relaxed"):
            fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    print("err", float((C2 - (A @ A) @ A).abs().max() / (A @ A @ A).abs().max()), flush=True)


if which == "A":
    s1, s2 = torch.cuda.Stream(priority=-1), torch.cuda.Stream()
    print("A: plain streams", flush=True)
    cap(lambda: forkjoin(s1, s2))
elif which == "B":
    ss = StreamSet(dev, reserve_cus=0)
    print("B: pipeline streams panel/update", flush=True)
    cap(lambda: forkjoin(ss.panel, ss.update[0]))
    print("B2: pipeline streams diag/panel", flush=True)
    cap(lambda: forkjoin(ss.diag, ss.panel))
else:
    N = 4096
    H = sl.HermitianMatrix(sl.Uplo.Lower, N, nb=512, device=dev)
    H.insertLocalTiles(device=dev)
    sl.generate_matrix(H, "poev", seed=3)
    buf = H.storage.local[H.storage.origin_slot]
    H0 = buf[:N, :N].clone()
    print("C: potrf graph, skipping", os.environ.get("SLATE_AMD_DEBUG_POTRF_SKIP"), flush=True)
    info = sl.potrf(H, {sl.Option.Lookahead: 1, sl.Option.UseGraph: True})
    torch.cuda.synchronize()
    L = torch.tril(buf[:N, :N])
    S = torch.tril(H0) + torch.tril(H0, -1).mT
    print("info", info, "err", float((L @ L.mT - S).norm() / S.norm()), flush=True)
print("probe2 done", which, flush=True)
