"""Eager vs Option.UseGraph one-rank potrf time for small orders (the
launch-bound regime a graph is for)."""
import time

import torch

import slate_amd as sl

dev = torch.device("cuda")
for n, nb in ((1024, 128), (2048, 256), (4096, 256), (8192, 512)):
    A = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb, device=dev)
    A.insertLocalTiles(device=dev)
    sl.generate_matrix(A, "poev", seed=1)
    buf = A.storage.local[A.storage.origin_slot]
    F0 = buf[:n, :n].clone()
    res = {}
    for mode in ("eager", "graph"):
        opts = {sl.Option.Lookahead: 1, sl.Option.UseGraph: mode == "graph"}
        ts = []
        for it in range(12):
            buf[:n, :n].copy_(F0)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            info = sl.potrf(A, opts)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
            if info != 0:
                print(f'n={n} nb={nb} {mode} iter {it}: info {info}', flush=True)
        res[mode] = sorted(ts[2:])[len(ts[2:]) // 2] * 1e3
    print(f"potrf n={n} nb={nb}: eager {res['eager']:.3f} ms, graph {res['graph']:.3f} ms", flush=True)
