"""Tester CLI (the reference's `test/test` TestSweeper driver, test/test.cc,
test/run_tests.py): parameter sweeps over routines with residual checks
and timings.

    python -m slate_amd.tester potrf --type d,z --dim 100:500:200 --nb 64 --uplo l,u
    torchrun --nproc-per-node 4 --master-addr 127.0.0.1 -m slate_amd.tester gemm --p 2 --q 2 --dim 1000

Options: --type s,d,c,z  --dim m[xn[xk]] or start:stop:step  --nb  --p --q
--target h|d  --check y|n  --uplo l,u  --trans n,t,c  --side l,r
--lookahead  --repeat.  One line per run: type, dims, nb, grid, error,
time, Gflop/s, status; exit status 1 if any check failed.
"""
from __future__ import annotations

import argparse
import itertools
import sys
import time

import torch

import slate_amd as sl
from slate_amd.core.enums import Diag, MethodEig, Norm, Op, Option, Side, Target, Uplo
from slate_amd.models.aux import allgather_dense as D

DT = {'s': torch.float32, 'd': torch.float64, 'c': torch.complex64, 'z': torch.complex128}
TOL = {'s': 3e-4, 'c': 3e-4, 'd': 1e-11, 'z': 1e-11}


def parse_dims(specs):
    out = []
    for spec in specs:
        for part in spec.split(","):
            fields = part.split("x")
            ranges = []
            for f in fields:
                if ":" in f:
                    a, b, c = (int(x) for x in (f.split(":") + ["1"])[:3])
                    ranges.append(list(range(a, b + 1, c)))
                else:
                    ranges.append([int(f)])
            while len(ranges) < 3:
                ranges.append(ranges[-1] if len(ranges) < 2 else ranges[0])
            n_runs = max(len(r) for r in ranges)
            for i in range(n_runs):
                out.append(tuple(r[min(i, len(r) - 1)] for r in ranges))
    return out


class Ctx:
    def __init__(self, a, t):
        self.a, self.t = a, t
        self.dt = DT[t]
        self.dev = torch.device("cuda", torch.cuda.current_device()) if a.target == 'd' else torch.device("cpu")
        self.opts = {Option.Target: Target.Devices if a.target == 'd' else Target.HostTask,
                     Option.Lookahead: a.lookahead}

    def mat(self, m, n, kind="rands", seed=1, cls=None, **kw):
        a = self.a
        if cls is None:
            M = sl.Matrix(m, n, nb=a.nb, p=a.p, q=a.q, dtype=self.dt, device=self.dev)
        elif cls is sl.HermitianMatrix:
            M = sl.HermitianMatrix(kw.get("uplo", Uplo.Lower), n, nb=a.nb, p=a.p, q=a.q, dtype=self.dt,
                                   device=self.dev)
        else:
            M = cls(**kw)
        M.insertLocalTiles(device=self.dev.index if self.dev.type == "cuda" else -1)
        sl.generate_matrix(M, kind, seed)
        return M

    def timed(self, fn):
        if self.dev.type == "cuda":
            torch.cuda.synchronize()
        sl.world().barrier()
        t0 = time.perf_counter()
        r = fn()
        if self.dev.type == "cuda":
            torch.cuda.synchronize()
        sl.world().barrier()
        return r, time.perf_counter() - t0


def _herm_full(A):
    from slate_amd.models.eig import _dense_hermitian
    return _dense_hermitian(A)


def _rel(R, scale):
    return float(R.abs().max()) / max(float(scale), 1e-300)


# ------------------------------------------------------------------ routines
def t_gemm(c, m, n, k, **p):
    A, B, C = c.mat(m, k, seed=1), c.mat(k, n, seed=2), c.mat(m, n, seed=3)
    Ad, Bd, Cd = D(A), D(B), D(C)
    _, t = c.timed(lambda: sl.gemm(1.0, A, B, 1.0, C, c.opts))
    err = _rel(D(C) - (Ad @ Bd + Cd), Ad.abs().max() * Bd.abs().max() * k) if c.a.check == 'y' else None
    return err, t, 2.0 * m * n * k


def t_herk(c, m, n, k, uplo=Uplo.Lower, **p):
    A = c.mat(n, k, seed=1)
    C = c.mat(n, n, seed=2, cls=sl.HermitianMatrix, uplo=uplo)
    Ad, Cf = D(A), _herm_full(C)
    _, t = c.timed(lambda: sl.herk(1.0, A, 1.0, C, c.opts))
    err = _rel(_herm_full(C) - (Ad @ Ad.mH + Cf), Ad.abs().max() ** 2 * k) if c.a.check == 'y' else None
    return err, t, 1.0 * n * n * k


def t_trsm(c, m, n, k, side=Side.Left, uplo=Uplo.Lower, **p):
    kk = m if side == Side.Left else n
    T = c.mat(kk, kk, seed=1)
    Td = D(T) + kk * torch.eye(kk, dtype=c.dt, device=D(T).device)
    sl.from_dense(T, Td)
    L = sl.TriangularMatrix(uplo, T)
    B = c.mat(m, n, seed=2)
    Bd = D(B)
    _, t = c.timed(lambda: sl.trsm(side, 1.0, L, B, c.opts))
    Tt = torch.tril(Td) if uplo == Uplo.Lower else torch.triu(Td)
    X = D(B)
    R = (Tt @ X - Bd) if side == Side.Left else (X @ Tt - Bd)
    return (_rel(R, Bd.abs().max() * kk) if c.a.check == 'y' else None), t, 1.0 * m * n * kk


def t_potrf(c, m, n, k, uplo=Uplo.Lower, **p):
    A = c.mat(n, n, "poev", 1, sl.HermitianMatrix, uplo=uplo)
    Af = _herm_full(A)
    info, t = c.timed(lambda: sl.potrf(A, c.opts))
    err = None
    if c.a.check == 'y':
        F = D(A)
        L = torch.tril(F) if uplo == Uplo.Lower else torch.triu(F).mH
        err = _rel(L @ L.mH - Af, Af.abs().max() * n)
    return err if info == 0 else float("inf"), t, n ** 3 / 3.0


def t_posv(c, m, n, k, uplo=Uplo.Lower, **p):
    A = c.mat(n, n, "poev", 1, sl.HermitianMatrix, uplo=uplo)
    B = c.mat(n, k, seed=2)
    Af, Bd = _herm_full(A), D(B)
    info, t = c.timed(lambda: sl.posv(A, B, c.opts))
    err = _rel(Af @ D(B) - Bd, Af.abs().max() * D(B).abs().max() * n) if c.a.check == 'y' else None
    return err if info == 0 else float("inf"), t, n ** 3 / 3.0 + 2.0 * n * n * k


def t_getrf(c, m, n, k, **p):
    A = c.mat(m, n, seed=1)
    Ad = D(A)
    piv = sl.Pivots()
    info, t = c.timed(lambda: sl.getrf(A, piv, c.opts))
    err = None
    if c.a.check == 'y':
        F = D(A)
        kk = min(m, n)
        L = torch.tril(F[:, :kk], -1) + torch.eye(m, kk, dtype=c.dt, device=F.device)
        U = torch.triu(F[:kk])
        PA = Ad.clone()
        for i, pv in enumerate(piv.ipiv.tolist()):
            if pv != i:
                PA[[i, pv]] = PA[[pv, i]]
        err = _rel(L @ U - PA, Ad.abs().max() * n)
    return err, t, 2.0 * n ** 3 / 3.0


def t_gesv(c, m, n, k, **p):
    A, B = c.mat(n, n, seed=1), c.mat(n, k, seed=2)
    Ad, Bd = D(A), D(B)
    info, t = c.timed(lambda: sl.gesv(A, sl.Pivots(), B, c.opts))
    X = D(B)
    err = _rel(Ad @ X - Bd, Ad.abs().max() * X.abs().max() * n) if c.a.check == 'y' else None
    return err, t, 2.0 * n ** 3 / 3.0 + 2.0 * n * n * k


def t_geqrf(c, m, n, k, **p):
    A = c.mat(m, n, seed=1)
    Ad = D(A)
    T = sl.TriangularFactors()
    _, t = c.timed(lambda: sl.geqrf(A, T, c.opts))
    err = None
    if c.a.check == 'y':
        Q = c.mat(m, m, "identity", 1)
        sl.unmqr(Side.Left, Op.NoTrans, A, T, Q, c.opts)
        kk = min(m, n)
        err = _rel(D(Q)[:, :kk] @ torch.triu(D(A))[:kk] - Ad, Ad.abs().max() * m)
    return err, t, 2.0 * m * n * n - 2.0 * n ** 3 / 3.0


def t_gels(c, m, n, k, **p):
    A, B = c.mat(m, n, seed=1), c.mat(max(m, n), k, seed=2)
    Ad, Bd = D(A), D(B)[:m].clone()
    _, t = c.timed(lambda: sl.gels(A, sl.TriangularFactors(), B, c.opts))
    X = D(B)[:n]
    ref = torch.linalg.lstsq(Ad.cpu(), Bd.cpu()).solution if m >= n else torch.linalg.pinv(Ad.cpu()) @ Bd.cpu()
    err = _rel(X.cpu() - ref, ref.abs().max() * max(m, n)) if c.a.check == 'y' else None
    return err, t, 2.0 * m * n * n


def t_heev(c, m, n, k, uplo=Uplo.Lower, **p):
    A = c.mat(n, n, seed=1, cls=sl.HermitianMatrix, uplo=uplo)
    Af = _herm_full(A).cpu()
    Z = c.mat(n, n, "zeros", 1)
    w, t = c.timed(lambda: sl.heev(A, None, Z, c.opts))
    Zd = D(Z).cpu()
    err = _rel(Af @ Zd - Zd * w.cpu().to(c.dt), Af.abs().max() * n) if c.a.check == 'y' else None
    return err, t, 4.0 * n ** 3 / 3.0


def t_svd(c, m, n, k, **p):
    A = c.mat(m, n, seed=1)
    Ad = D(A).cpu()
    kk = min(m, n)
    U, VH = c.mat(m, kk, "zeros"), c.mat(kk, n, "zeros")
    s, t = c.timed(lambda: sl.svd(A, None, U, VH, c.opts))
    err = _rel(D(U).cpu() @ torch.diag(s.cpu().to(c.dt)) @ D(VH).cpu() - Ad, Ad.abs().max() * max(m, n)) \
        if c.a.check == 'y' else None
    return err, t, 4.0 * m * n * n


def t_norm(c, m, n, k, **p):
    A = c.mat(m, n, seed=1)
    Ad = D(A)
    v, t = c.timed(lambda: sl.norm(Norm.Fro, A, c.opts))
    return abs(float(v) - float(torch.linalg.norm(Ad))) / float(torch.linalg.norm(Ad)), t, 2.0 * m * n


def t_gesv_mixed(c, m, n, k, **p):
    if c.t not in ('d', 'z'):
        return None, 0.0, 0.0
    A, B = c.mat(n, n, "rand_dominant", 1), c.mat(n, k, seed=2)
    X = c.mat(n, k, "zeros")
    Ad, Bd = D(A), D(B)
    r, t = c.timed(lambda: sl.gesv_mixed(A, sl.Pivots(), B, X, c.opts))
    err = _rel(Ad @ D(X) - Bd, Ad.abs().max() * D(X).abs().max() * n) if c.a.check == 'y' else None
    return err, t, 2.0 * n ** 3 / 3.0


def t_hesv(c, m, n, k, **p):
    A, B = c.mat(n, n, seed=1, cls=sl.HermitianMatrix), c.mat(n, k, seed=2)
    Af, Bd = _herm_full(A), D(B)
    _, t = c.timed(lambda: sl.hesv(A, sl.Pivots(), None, None, None, B, c.opts))
    err = _rel(Af @ D(B) - Bd, Af.abs().max() * D(B).abs().max() * n) if c.a.check == 'y' else None
    return err, t, n ** 3 / 3.0


ROUTINES = {"gemm": t_gemm, "herk": t_herk, "syrk": t_herk, "trsm": t_trsm, "potrf": t_potrf,
            "posv": t_posv, "getrf": t_getrf, "gesv": t_gesv, "geqrf": t_geqrf, "gels": t_gels,
            "heev": t_heev, "syev": t_heev, "svd": t_svd, "norm": t_norm, "genorm": t_norm,
            "gesv_mixed": t_gesv_mixed, "hesv": t_hesv, "sysv": t_hesv}


def main(argv=None):
    ap = argparse.ArgumentParser(prog="slate_amd.tester")
    ap.add_argument("routine", choices=sorted(ROUTINES))
    ap.add_argument("--type", default="d")
    ap.add_argument("--dim", action="append", default=[])
    ap.add_argument("--nb", default="256")
    ap.add_argument("--p", type=int, default=1)
    ap.add_argument("--q", type=int, default=1)
    ap.add_argument("--target", default="d" if torch.cuda.is_available() else "h")
    ap.add_argument("--check", default="y")
    ap.add_argument("--uplo", default="l")
    ap.add_argument("--side", default="l")
    ap.add_argument("--lookahead", type=int, default=1)
    ap.add_argument("--repeat", type=int, default=1)
    a = ap.parse_args(argv)
    comm = sl.init()
    if a.p * a.q != comm.size:
        a.p, a.q = 1, comm.size
    dims = parse_dims(a.dim or ["100:300:100"])
    fn = ROUTINES[a.routine]
    fails = 0
    if comm.rank == 0:
        print(f"{'type':>4} {'m':>6} {'n':>6} {'k':>6} {'nb':>5} {'grid':>6} {'uplo':>4} {'error':>10} "
              f"{'time(s)':>9} {'Gflop/s':>9}  status", flush=True)
    for t, (m, n, k), nb, up, sd in itertools.product(a.type.split(","), dims, a.nb.split(","),
                                                      a.uplo.split(","), a.side.split(",")):
        a.nb = int(nb)
        ctx = Ctx(a, t)
        uplo = Uplo.Lower if up.lower() == 'l' else Uplo.Upper
        side = Side.Left if sd.lower() == 'l' else Side.Right
        for _ in range(a.repeat):
            try:
                err, tm, fl = fn(ctx, m, n, k, uplo=uplo, side=side)
                ok = err is None or err < TOL[t] * (10 if a.routine in ("heev", "svd", "gels") else 1)
            except Exception as e:  # noqa: BLE001
                err, tm, fl, ok = float("nan"), 0.0, 0.0, False
                if comm.rank == 0:
                    print(f"  error: {e}", file=sys.stderr)
            fails += 0 if ok else 1
            if comm.rank == 0:
                es = "-" if err is None else f"{err:10.2e}"
                gf = fl / tm / 1e9 if tm > 0 else 0.0
                print(f"{t:>4} {m:>6} {n:>6} {k:>6} {a.nb:>5} {f'{a.p}x{a.q}':>6} {up:>4} {es:>10} {tm:9.4f} "
                      f"{gf:9.1f}  {'pass' if ok else 'FAILED'}", flush=True)
    if comm.rank == 0:
        print("All tests passed." if fails == 0 else f"{fails} tests FAILED.", flush=True)
    sl.finalize()
    return 1 if fails else 0


if __name__ == "__main__":
    sys.exit(main())
