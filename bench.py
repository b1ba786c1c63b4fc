#!/usr/bin/env python3
"""Headline benchmark: distributed dpotrf (Cholesky), n=32768, nb=512, fp64.

Metric (BASELINE.json): GFLOP/s and % of fp64 peak for dpotrf/dgetrf at
n=32768 nb=512 on 1/2/4/8 MI355X.  One "step" = one full factorization of a
freshly restored SPD matrix (the restore is a device-to-device copy of the
local buffer and IS inside the timed region -- conservative).  Flops use the
LAPACK/SLATE convention n^3/3 + n^2/2 + n/6 (docs/latex/flops.tex:103).

Launch: python bench.py [--gpus N --steps K --warmup W]
        N>1: one process per GPU, RCCL over xGMI -- either under an external
        torchrun (WORLD_SIZE set, must equal N) or, without one, bench.py
        starts the N ranks itself before any GPU call (_self_launch).
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


class _DistVec:
    """Matrix-vector products with a block-cyclic local buffer, for the
    correctness check after the timed region (no gather of the matrix: each
    rank multiplies its local block, one all-reduce of an n-vector)."""

    def __init__(self, M, comm):
        st = M.storage
        bc = st.bc
        self.comm = comm
        self.dev = st.local[st.origin_slot].device
        lr = torch.arange(bc.mloc, device=self.dev)
        lc = torch.arange(bc.nloc, device=self.dev)
        self.gr = ((lr // bc.mb) * bc.p + bc.pr) * bc.mb + lr % bc.mb
        self.gc = ((lc // bc.nb) * bc.q + bc.pc) * bc.nb + lc % bc.nb
        self.m, self.n = st.m, st.n
        self.mloc, self.nloc = bc.mloc, bc.nloc

    def local(self, buf):
        return buf[:self.mloc, :self.nloc]

    def _sum(self, y):
        if self.comm.size > 1:
            self.comm.allreduce(y)
        return y

    def mv(self, F, v):
        """y = F v (F: masked local block of an m x n matrix, v: n)."""
        y = torch.zeros(self.m, dtype=v.dtype, device=v.device)
        if F.numel():
            y[self.gr] = F @ v[self.gc]
        return self._sum(y)

    def mvT(self, F, v):
        """w = F^T v (v: m)."""
        w = torch.zeros(self.n, dtype=v.dtype, device=v.device)
        if F.numel():
            w[self.gc] = F.mT @ v[self.gr]
        return self._sum(w)

    def fro2(self, F):
        t = (F * F).sum().reshape(1)
        return float(self._sum(t).item())


def _residual(args, A, A0, piv, comm, extra=None):
    """Backward error of the last factorization (outside the timed region),
    computed on the grid: a random vector v is pushed through the factors
    and through the saved input.  Tester-style checks (reference
    test/test_posv.cc:304-345, test_gesv.cc:332-377):
      potrf  ||L L^T v - A v|| / (||A|| ||v|| n)
      getrf  ||L U v - P A v|| / (||A|| ||v|| n)
      geqrf  ||R^T R v - A^T A v|| / (||A||^2 ||v|| n)     (Q-free)
      gemm   ||C v - A (B v)|| / (||A (B v)|| (sqrt(n) + 2))   (test_gemm.cc:191-207)
    Must be O(eps): bench.py exits non-zero above 3 eps (the reference
    tester's default tolerance factor).  Returns (normalised, raw): raw is
    the same quotient WITHOUT the 1/n (with the n a
    systematic 1e3 eps error would still pass); potrf, backward stable with
    no growth, is also gated on raw <= 3 eps."""
    D = _DistVec(A, comm)
    st = A.storage
    F = D.local(st.local[st.origin_slot])
    F0 = D.local(A0)
    gr, gc = D.gr[:, None], D.gc[None, :]
    g = torch.Generator(device="cpu").manual_seed(5)
    n = st.n
    if args.routine == "potrf":
        v = torch.rand(n, 1, generator=g, dtype=torch.float64).to(D.dev)[:, 0]
        L = torch.where(gr >= gc, F, torch.zeros((), dtype=F.dtype, device=F.device))
        y = D.mv(L, D.mvT(L, v))
        Lo = torch.where(gr >= gc, F0, torch.zeros((), dtype=F0.dtype, device=F0.device))
        So = torch.where(gr > gc, F0, torch.zeros((), dtype=F0.dtype, device=F0.device))
        sv = D.mv(Lo, v) + D.mvT(So, v)
        nA = (D.fro2(Lo) + D.fro2(So)) ** 0.5
        r = (y - sv).norm() / (nA * v.norm() * n)
    elif args.routine == "getrf":
        v = torch.rand(n, 1, generator=g, dtype=torch.float64).to(D.dev)[:, 0]
        z = torch.zeros((), dtype=F.dtype, device=F.device)
        U = torch.where(gr <= gc, F, z)
        Ls = torch.where(gr > gc, F, z)
        u = D.mv(U, v)
        y = D.mv(Ls, u) + u
        a = D.mv(F0, v).cpu()
        perm = list(range(n))
        for i, j in enumerate(piv.ipiv.tolist()):      # LAPACK-style sequential swaps
            perm[i], perm[j] = perm[j], perm[i]
        pa = a[torch.as_tensor(perm)].to(D.dev)
        r = (y - pa).norm() / (D.fro2(F0) ** 0.5 * v.norm() * n)
    elif args.routine == "geqrf":
        v = torch.rand(n, 1, generator=g, dtype=torch.float64).to(D.dev)[:, 0]
        R = torch.where(gr <= gc, F, torch.zeros((), dtype=F.dtype, device=F.device))
        z1 = D.mvT(F0, D.mv(F0, v))
        z2 = D.mvT(R, D.mv(R, v))
        r = (z1 - z2).norm() / (D.fro2(F0) * v.norm() * n)
    elif args.routine == "gemm":
        Bm, Cm = extra
        DB = _DistVec(Bm, comm)
        v = torch.rand(n, 1, generator=g, dtype=torch.float64).to(D.dev)[:, 0]
        FB = DB.local(Bm.storage.local[Bm.storage.origin_slot])
        FC = DB.local(Cm.storage.local[Cm.storage.origin_slot])
        y = DB.mv(FC, v)
        x = D.mv(F0, DB.mv(FB, v))
        r = (y - x).norm() / (x.norm() * (n ** 0.5 + 2))
    else:
        return None, None
    raw = float(r) * (1 if args.routine == "gemm" else n)
    return float(f"{float(r):.3e}"), float(f"{raw:.3e}")


def _main_native(args):
    """bench.py --impl native: the same step / timing / JSON contract through
    libslate_amd_native.so.  This process never touches the GPU; it starts
    slate_amd/bench_native as a child with the same RANK / WORLD_SIZE /
    MASTER_* environment (the native runtime bootstraps RCCL itself on
    MASTER_PORT + 1) and rank 0 prints the JSON line."""
    import re
    import subprocess
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.routine not in ("potrf", "getrf", "gemm", "geqrf"):
        raise SystemExit("--impl native: potrf, getrf, gemm or geqrf")
    p, q = grid_for(world, args.routine) if args.grid is None else map(int, args.grid.lower().split("x"))
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "slate_amd", "bench_native")
    cmd = [exe, args.routine, str(args.n), str(args.nb), str(p), str(q), str(args.lookahead), str(args.warmup),
           str(args.steps), str(args.check), str(args.m or args.n)]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        print(r.stdout, file=sys.stderr, flush=True)
        raise SystemExit(r.returncode)
    if rank != 0:
        return
    m = re.search(r"RESULT ms_per_step=(\S+) info=(\S+) resid=(\S+) transport=(\S+)", r.stdout)
    ms, info, resid, transport = float(m.group(1)), int(m.group(2)), float(m.group(3)), m.group(4)
    fl = flops(args.routine, args.n, args.m)
    gflops = fl / (ms * 1e-3) / 1e9
    tol = 3 * 2.0 ** -52
    resid = resid if args.check else None
    out = {
        "metric": (f"d{args.routine} GFLOP/s (m={args.m or args.n}, n={args.n}, nb={args.nb})"
                   if args.routine == "geqrf" else f"d{args.routine} GFLOP/s (n={args.n}, nb={args.nb})"),
        "value": round(gflops, 2),
        "unit": "GFLOP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "fp64",
        "data": "synthetic (Philox SPD/rand matrix generated on device)",
        "impl": f"native C++ library (libslate_amd_native.so, transport {transport})",
        "pct_fp64_peak": round(100 * gflops / 1e3 / (FP64_PEAK_TF * world), 2),
        "info_ok": info == 0,
        "residual": resid,
        "residual_ok": None if resid is None else bool(resid <= tol),
        "config": {"model": f"d{args.routine} n={args.n} nb={args.nb}", "global_batch": 1, "seq_len": args.n,
                   "n": args.n, "nb": args.nb, "grid": f"{p}x{q}", "lookahead": args.lookahead,
                   "parallelism": f"2d-block-cyclic {p}x{q}"},
    }
    print(json.dumps(out), flush=True)
    if info != 0 or (resid is not None and not resid <= tol):
        print(f"bench: FAILED correctness check (info={info}, residual={resid}, tol={tol:.2e})",
              file=sys.stderr, flush=True)
        sys.exit(1)


def _free_port_pair():
    """A port P with P and P + 1 both free on 127.0.0.1."""
    import socket
    for _ in range(64):
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        try:
            with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
                s.bind(("127.0.0.1", port + 1))
            return port
        except OSError:
            continue
    raise SystemExit("bench: no free port pair on 127.0.0.1")


def _self_launch(nproc):
    """``--gpus N`` (N > 1) started without a launcher: start N ranks here,
    one process per GPU (rank r -> LOCAL_RANK r -> GPU r), the way the
    reference's tester is started per rank by mpirun
    (/root/reference/test/run_tests.py:171-175).  This parent never touches
    the GPU (no HIP call happens before or after the spawn: torch is only
    imported) and never exec()s -- the ranks are children of a
    torch.distributed.run child; rank 0's JSON line goes straight to our
    stdout, and any rank failing makes this process exit non-zero.
    MASTER_PORT + 1 stays free for the native runtime's own bootstrap
    (--impl native)."""
    import subprocess
    port = _free_port_pair()
    cmd =[sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    r = subprocess.run(cmd, env=env)
    if r.returncode != 0:
        print(f"bench: {nproc}-rank launch failed (exit {r.returncode})", file=sys.stderr, flush=True)
    sys.exit(r.returncode)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    # --size / --rows: the same, usable after `python -m torch.distributed.run ... bench.py`
    # (its parser takes --n / --m for ambiguous prefixes of its own options)
    ap.add_argument("--n", "--size", dest="n", type=int, default=32768)
    ap.add_argument("--m", "--rows", dest="m", type=int, default=None)
    ap.add_argument("--nb", type=int, default=None, help="tile size (default: 256 for geqrf, 512 otherwise -- BASELINE)")
    ap.add_argument("--routine", default="potrf", choices=["potrf", "getrf", "gemm", "geqrf", "heev"])
    ap.add_argument("--vectors", type=int, default=1, help="heev: 1 = eigenvectors (dsyevd), 0 = values only")
    ap.add_argument("--band", type=int, default=0, help="heev: stage-1 bandwidth (default min(nb, 64))")
    ap.add_argument("--lookahead", type=int, default=1)
    ap.add_argument("--method", default="pp", choices=["pp", "calu", "nopiv"], help="getrf: pivoting method")
    ap.add_argument("--grid", default=None, help="PxQ override")
    ap.add_argument("--check", type=int, default=1, help="residual check after timing (0 = skip)")
    ap.add_argument("--impl", default="python", choices=["python", "native"],
                    help="native: the Python-free C++ library (slate_amd/bench_native, one child per rank)")
    args = ap.parse_args()
    if args.nb is None:
        args.nb = 256 if args.routine == "geqrf" else 512
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return _self_launch(args.gpus)
    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    if env_world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE {env_world} (one rank per GPU)")
    if args.impl == "native":
        return _main_native(args)
    # No GPU_MAX_HW_QUEUES override: a process drives the panel, diag and
    # update streams plus the caller's -- the box default of 4 hardware
    # queues.  RCCL adds none: torch runs every synchronous collective on
    # the issuing stream (profiles/r4/nccl_stream_probe.txt) and each
    # communicator is issued from one stream only (tests/test_dist_gpu.py).

    import slate_amd as sl
    comm = sl.init()
    world = comm.size
    rank = comm.rank
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but the communicator has {world} ranks")
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
    t_host = time.perf_counter() - t0     # host time to issue the K steps (drivers return after their final info read)
    comm.barrier()
    sync()
    dt = time.perf_counter() - t0
    dt_max = comm.allreduce_scalar(dt, "max") if world > 1 else dt
    host_max = comm.allreduce_scalar(t_host, "max") if world > 1 else t_host
    extra = (B, C) if args.routine == "gemm" else None
    resid, resid_raw = _residual(args, A, backup, locals().get("piv"), comm, extra) if args.check else (None, None)
    tol = 3 * 2.0 ** -52                 # reference tester default: tol 3 x eps
    raw_bad = args.routine == "potrf" and resid_raw is not None and not resid_raw <= tol
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
            "residual_ok": None if resid is None else bool(resid <= tol and not raw_bad),
            "residual_raw": resid_raw,
            "host_ms_per_step": round(host_max / args.steps * 1e3, 3),
            "config": {"model": f"d{args.routine} n={n} nb={nb}", "global_batch": 1, "seq_len": n,
                       "n": n, "nb": nb, "grid": f"{p}x{q}", "lookahead": args.lookahead,
                       "parallelism": f"2d-block-cyclic {p}x{q}"},
        }
        print(json.dumps(out), flush=True)
    sl.finalize()
    bad = (not ok) or (resid is not None and not resid <= tol) or raw_bad
    if bad:
        print(f"bench: FAILED correctness check (info_ok={ok}, residual={resid}, raw={resid_raw}, tol={tol:.2e})",
              file=sys.stderr, flush=True)
        sys.exit(1)


if __name__ == "__main__":
    main()
