#!/usr/bin/env python3
"""Headline benchmark: distributed dpotrf (Cholesky), n=32768, nb=512, fp64.

Metric (BASELINE.json): GFLOP/s and % of fp64 peak for dpotrf/dgetrf at
n=32768 nb=512 on 1/2/4/8 MI355X.  One "step" = one full factorization of a
freshly restored SPD matrix (the restore is a device-to-device copy of the
local buffer and IS inside the timed region -- conservative).  Flops use the
LAPACK/SLATE convention n^3/3 + n^2/2 + n/6 (docs/latex/flops.tex:103).

Launch: python bench.py [--gpus N --steps K --warmup W]
        (N>1 via torchrun: one process per GPU, RCCL over xGMI)
Grid:   1x1, 1x2, 2x2, 2x4 for 1, 2, 4, 8 GPUs (BASELINE: 2x4 at 8).
Data:   synthetic SPD matrix (Hermitian rands + n*I, Philox, generated on
        device); random-init of the named config, no external data.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

FP64_PEAK_TF = 78.6   # MI355X fp64 (vector == matrix) per GPU, vendor spec


def flops(routine, n, m=None):
    if routine == "potrf":
        return n ** 3 / 3 + n ** 2 / 2 + n / 6
    if routine == "getrf":
        return 2 * n ** 3 / 3 - n ** 2 / 2 + 5 * n / 6
    if routine == "gemm":
        return 2.0 * n ** 3
    if routine == "geqrf":
        m = m or n
        return 2 * m * n ** 2 + m * n - 2 * n ** 3 / 3 + n ** 2 + 14 * n / 3
    if routine == "heev":
        return 4 * n ** 3 / 3          # sytrd (stage-1 equivalent) flops, docs/latex/flops.tex:268
    raise ValueError(routine)


def grid_for(n, routine="potrf"):
    """Default process grid per GPU count.  potrf/getrf/gemm: as square as
    possible with q >= p (BASELINE: 2x4 at 8 GPUs); geqrf (tall-skinny QR,
    m = 8n): one process column (p = N) -- the TSQR tree spans all GPUs and
    the trailing update needs no row broadcast."""
    if routine == "geqrf":
        return (n, 1)
    return {1: (1, 1), 2: (1, 2), 4: (2, 2), 8: (2, 4)}.get(n, (1, n))


def _residual(args, A, A0, piv):
    """Backward error of the last factorization (outside the timed region),
    one rank only.  Mirrors the reference tester's checks
    (test/test_posv.cc:304-345, test_gesv.cc:332-377): a random right-hand
    side is pushed through the factors and ||A0 x - b|| / (||A0|| ||x|| n)
    is reported; it must be O(eps)."""
    F = A.storage.local[A.storage.origin_slot]
    m, n = F.shape[0], F.shape[1]
    g = torch.Generator(device=F.device).manual_seed(5)
    if args.routine == "potrf":
        L = torch.tril(F[:n, :n])
        S = torch.tril(A0[:n, :n])
        S = S + torch.tril(S, -1).mT
        b = torch.rand(n, 1, dtype=F.dtype, device=F.device, generator=g)
        y = torch.linalg.solve_triangular(L, b, upper=False)
        x = torch.linalg.solve_triangular(L.mT, y, upper=True)
        r = (S @ x - b).norm() / (S.norm() * x.norm() * n)
    elif args.routine == "getrf":
        b = torch.rand(n, 1, dtype=F.dtype, device=F.device, generator=g)
        perm = list(range(n))
        for i, j in enumerate(piv.ipiv.tolist()):     # LAPACK-style sequential swaps
            perm[i], perm[j] = perm[j], perm[i]
        pb = b[torch.as_tensor(perm, device=F.device)]
        Lu = torch.tril(F[:n, :n], -1) + torch.eye(n, dtype=F.dtype, device=F.device)
        y = torch.linalg.solve_triangular(Lu, pb, upper=False)
        x = torch.linalg.solve_triangular(torch.triu(F[:n, :n]), y, upper=True)
        r = (A0[:n, :n] @ x - b).norm() / (A0[:n, :n].norm() * x.norm() * n)
    elif args.routine == "geqrf":
        R = torch.triu(F[:n, :n])
        # ||R^T R - A^T A|| / (||A||^2 n): Q-free backward-error proxy
        r = (R.mT @ R - A0.mT @ A0).norm() / (A0.norm() ** 2 * n)
    else:
        return None
    return float(f"{r.item():.3e}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    # --size / --rows: the same, usable after `python -m torch.distributed.run ... bench.py`
    # (its parser takes --n / --m for ambiguous prefixes of its own options)
    ap.add_argument("--n", "--size", dest="n", type=int, default=32768)
    ap.add_argument("--m", "--rows", dest="m", type=int, default=None)
    ap.add_argument("--nb", type=int, default=512)
    ap.add_argument("--routine", default="potrf", choices=["potrf", "getrf", "gemm", "geqrf", "heev"])
    ap.add_argument("--vectors", type=int, default=1, help="heev: 1 = eigenvectors (dsyevd), 0 = values only")
    ap.add_argument("--band", type=int, default=0, help="heev: stage-1 bandwidth (default min(nb, 64))")
    ap.add_argument("--lookahead", type=int, default=1)
    ap.add_argument("--method", default="pp", choices=["pp", "calu", "nopiv"], help="getrf: pivoting method")
    ap.add_argument("--grid", default=None, help="PxQ override")
    ap.add_argument("--check", type=int, default=1, help="residual check after timing (1 rank)")
    args = ap.parse_args()

    import slate_amd as sl
    comm = sl.init()
    world = comm.size
    rank = comm.rank
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    p, q = grid_for(world, args.routine) if args.grid is None else map(int, args.grid.lower().split("x"))
    gpu = torch.cuda.is_available()
    dev = torch.device("cuda", torch.cuda.current_device()) if gpu else torch.device("cpu")
    sync = torch.cuda.synchronize if gpu else (lambda: None)
    n, nb = args.n, args.nb
    opts = {sl.Option.Lookahead: args.lookahead,
            sl.Option.Target: sl.Target.Devices if gpu else sl.Target.HostTask}

    if args.routine == "potrf":
        A = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb, p=p, q=q, device=dev)
        A.insertLocalTiles(device=dev)
        sl.generate_matrix(A, "poev", seed=7)
        run = lambda: sl.potrf(A, opts)
    elif args.routine == "getrf":
        A = sl.Matrix(n, n, nb=nb, p=p, q=q, device=dev)
        A.insertLocalTiles(device=dev)
        sl.generate_matrix(A, "rands", seed=7)
        piv = sl.Pivots()
        opts[sl.Option.MethodLU] = {"pp": sl.MethodLU.PartialPiv, "calu": sl.MethodLU.CALU,
                                    "nopiv": sl.MethodLU.NoPiv}[args.method]
        run = lambda: sl.getrf(A, piv, opts)
    elif args.routine == "geqrf":
        m = args.m or n
        A = sl.Matrix(m, n, nb=nb, p=p, q=q, device=dev)
        A.insertLocalTiles(device=dev)
        sl.generate_matrix(A, "rands", seed=7)
        T = sl.TriangularFactors()
        run = lambda: sl.geqrf(A, T, opts)
    elif args.routine == "heev":
        A = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb, p=p, q=q, device=dev)
        A.insertLocalTiles(device=dev)
        sl.generate_matrix(A, "rands", seed=7)
        Zm = None
        if args.vectors:
            Zm = sl.Matrix(n, n, nb=nb, p=p, q=q, device=dev)
            Zm.insertLocalTiles(device=dev)
        hopts = dict(opts)
        if args.band:
            hopts[sl.Option.InnerBlocking] = args.band
        run = lambda: sl.heev(A, None, Zm, hopts)
    else:
        A = sl.Matrix(n, n, nb=nb, p=p, q=q, device=dev)
        A.insertLocalTiles(device=dev)
        sl.generate_matrix(A, "rands", seed=7)
        B = sl.Matrix(n, n, nb=nb, p=p, q=q, device=dev); B.insertLocalTiles(device=dev)
        sl.generate_matrix(B, "rands", seed=8)
        C = sl.Matrix(n, n, nb=nb, p=p, q=q, device=dev); C.insertLocalTiles(device=dev)
        run = lambda: sl.gemm(1.0, A, B, 0.0, C, opts)
    local = A.storage.local[A.storage.origin_slot]
    backup = local.clone()

    def step():
        local.copy_(backup)          # restore the input (inside the timed region)
        A.storage.mark_local_modified(A.storage.origin_slot)
        return run()

    for _ in range(args.warmup):
        info = step()
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        info = step()
    comm.barrier()
    sync()
    dt = time.perf_counter() - t0
    dt_max = comm.allreduce_scalar(dt, "max") if world > 1 else dt
    resid = _residual(args, A, backup, locals().get("piv")) if (world == 1 and args.check) else None
    fl = flops(args.routine, n, args.m)
    gflops = fl * args.steps / dt_max / 1e9
    ok = (info == 0) if isinstance(info, int) else True
    if rank == 0 and args.routine == "heev":
        # BASELINE: time to solution (dsyevd n=16384 nb=256)
        out = {
            "metric": f"dsyev{'d' if args.vectors else ''} time to solution (n={n}, nb={nb})",
            "value": round(dt_max / args.steps, 4),
            "unit": "s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt_max / args.steps * 1e3, 3),
            "higher_is_better": False,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "fp64",
            "data": "synthetic (Philox random Hermitian matrix generated on device)",
            "gflops_4n3_3": round(gflops, 2),
            "config": {"model": f"dsyevd n={n} nb={nb}", "global_batch": 1, "seq_len": n, "n": n, "nb": nb,
                       "grid": f"{p}x{q}", "parallelism": f"2d-block-cyclic {p}x{q}"},
        }
        print(json.dumps(out), flush=True)
    elif rank == 0:
        out = {
            "metric": (f"d{args.routine} GFLOP/s (m={args.m or n}, n={n}, nb={nb})" if args.routine == "geqrf"
                       else f"d{args.routine} GFLOP/s (n={n}, nb={nb})"),
            "value": round(gflops, 2),
            "unit": "GFLOP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt_max / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "fp64",
            "data": "synthetic (Philox SPD/rand matrix generated on device)",
            "pct_fp64_peak": round(100 * gflops / 1e3 / (FP64_PEAK_TF * world), 2),
            "info_ok": bool(ok),
            "residual": resid,
            "config": {"model": f"d{args.routine} n={n} nb={nb}", "global_batch": 1, "seq_len": n,
                       "n": n, "nb": nb, "grid": f"{p}x{q}", "lookahead": args.lookahead,
                       "parallelism": f"2d-block-cyclic {p}x{q}"},
        }
        print(json.dumps(out), flush=True)
    sl.finalize()


if __name__ == "__main__":
    main()
