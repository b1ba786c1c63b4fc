"""Multi-rank device-path check on a ONE-GPU box: 2 (or 4) ranks share
cuda:0 over gloo (tensors staged through the host by Comm._prep), so the
distributed drivers' device code (panel broadcasts, row exchanges,
lookahead, masked updates) runs on the gfx950 kernels for p x q grids.
Performance is meaningless here; correctness is the point.

    python tools/check_dist_gpu.py [nprocs]
"""
import os
import socket
import sys
import time
import traceback

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def work(rank, size, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(size),
                      LOCAL_RANK="0")
    try:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=size)
        torch.cuda.set_device(0)
        import slate_amd as sl
        from slate_amd.models.aux import allgather_dense as D
        from slate_amd.models.eig import _dense_hermitian
        dev = torch.device("cuda", 0)
        grids = [(2, 1), (1, 2)] if size == 2 else [(2, 2), (4, 1), (1, 4)]
        out = []
        for (p, qq) in grids:
            n, nb = 1000, 128
            opts = {sl.Option.Target: sl.Target.Devices, sl.Option.Lookahead: 1}
            # potrf
            A = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb, p=p, q=qq, device=dev)
            A.insertLocalTiles(device=0)
            sl.generate_matrix(A, "poev", 3)
            Af = _dense_hermitian(A)
            t0 = time.perf_counter()
            info = sl.potrf(A, opts)
            torch.cuda.synchronize()
            L = torch.tril(D(A))
            e1 = ((L @ L.mH - Af).abs().max() / (Af.abs().max() * n)).item()
            # getrf / gesv
            M = sl.Matrix(n, n, nb=nb, p=p, q=qq, device=dev)
            M.insertLocalTiles(device=0)
            sl.generate_matrix(M, "rands", 4)
            Md = D(M).clone()
            B = sl.Matrix(n, 3, nb=nb, p=p, q=qq, device=dev)
            B.insertLocalTiles(device=0)
            sl.generate_matrix(B, "rands", 5)
            Bd = D(B).clone()
            info2 = sl.gesv(M, sl.Pivots(), B, opts)
            e2 = ((Md @ D(B) - Bd).abs().max() / (Md.abs().max() * D(B).abs().max() * n)).item()
            # gemm
            X = sl.Matrix(n, 700, nb=nb, p=p, q=qq, device=dev)
            Y = sl.Matrix(700, 600, nb=nb, p=p, q=qq, device=dev)
            Z = sl.Matrix(n, 600, nb=nb, p=p, q=qq, device=dev)
            for i, W in enumerate((X, Y, Z)):
                W.insertLocalTiles(device=0)
                sl.generate_matrix(W, "rands", 10 + i)
            Xd, Yd, Zd = D(X), D(Y), D(Z)
            sl.gemm(1.0, X, Y, 1.0, Z, opts)
            e3 = ((D(Z) - (Xd @ Yd + Zd)).abs().max() / (Xd.abs().max() * Yd.abs().max() * 700)).item()
            # geqrf
            G = sl.Matrix(n, 600, nb=nb, p=p, q=qq, device=dev)
            G.insertLocalTiles(device=0)
            sl.generate_matrix(G, "rands", 6)
            Gd = D(G).clone()
            T = sl.TriangularFactors()
            sl.geqrf(G, T, opts)
            Q = sl.Matrix(n, n, nb=nb, p=p, q=qq, device=dev)
            Q.insertLocalTiles(device=0)
            sl.set(0.0, 1.0, Q)
            sl.unmqr(sl.Side.Left, sl.Op.NoTrans, G, T, Q, opts)
            e4 = ((D(Q)[:, :600] @ torch.triu(D(G))[:600] - Gd).abs().max() / (Gd.abs().max() * n)).item()
            dt = time.perf_counter() - t0
            out.append(f"grid {p}x{qq}: potrf info={info} err={e1:.2e} | gesv info={info2} err={e2:.2e} | "
                       f"gemm err={e3:.2e} | geqrf err={e4:.2e} | {dt:.1f}s")
            assert info == 0 and info2 == 0 and e1 < 1e-14 and e2 < 1e-13 and e3 < 1e-14 and e4 < 1e-13, out[-1]
        dist.destroy_process_group()
        q.put((rank, out, None))
    except BaseException:  # noqa: BLE001
        q.put((rank, None, traceback.format_exc()))


if __name__ == "__main__":
    size = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=work, args=(r, size, port, q)) for r in range(size)]
    for p in ps:
        p.start()
    ok = True
    for _ in range(size):
        r, out, err = q.get(timeout=900)
        if err:
            ok = False
            print(f"rank {r} FAILED:\n{err}", flush=True)
        elif r == 0:
            print("\n".join(out), flush=True)
    for p in ps:
        p.join(timeout=60)
    sys.exit(0 if ok else 1)
