"""Tester CLI (the reference's `test/test` TestSweeper driver, test/test.cc,
test/run_tests.py): parameter sweeps over routines with residual checks
and timings.

    python -m slate_amd.tester potrf --type d,z --dim 100:500:200 --nb 64 --uplo l,u
    torchrun --nproc-per-node 4 --master-addr 127.0.0.1 -m slate_amd.tester gemm --p 2 --q 2 --dim 1000

Options: --type s,d,c,z  --dim m[xn[xk]] or start:stop:step  --nb  --p --q
--target h|d  --check y|n  --uplo l,u  --trans n,t,c  --side l,r
--lookahead  --repeat.  One line per run: type, dims, nb, grid, error,
time, Gflop/s, % of the MI355X dense peak of all ranks (device target),
status; exit status 1 if any check failed.  Routines (test/test.cc
families): BLAS-3 gemm herk/syrk her2k/syr2k hemm/symm trmm trsm;
Cholesky potrf potrs posv potri trtri posv_mixed; LU getrf getrs gesv
getri gesv_nopiv gesv_tntpiv/calu gesv_rbt gesv_mixed gesv_mixed_gmres;
band gbsv pbsv gbmm hbmm tbsm; QR/LQ geqrf unmqr gelqf cholqr gels;
eigen/SVD heev/syev heev_vals hegv/sygv svd svd_vals; indefinite
hesv/sysv; aux norm colnorms add redistribute gecondest pocondest
trcondest matgen.
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


def _herm_mat(c, n, uplo, kind="rands", seed=1):
    return c.mat(n, n, kind, seed, sl.HermitianMatrix, uplo=uplo)


def t_her2k(c, m, n, k, uplo=Uplo.Lower, **p):
    A, B = c.mat(n, k, seed=1), c.mat(n, k, seed=2)
    C = _herm_mat(c, n, uplo, seed=3)
    Ad, Bd, Cf = D(A), D(B), _herm_full(C)
    _, t = c.timed(lambda: sl.her2k(1.0, A, B, 1.0, C, c.opts))
    ref = Ad @ Bd.mH + Bd @ Ad.mH + Cf
    err = _rel(_herm_full(C) - ref, Ad.abs().max() * Bd.abs().max() * k) if c.a.check == 'y' else None
    return err, t, 2.0 * n * n * k


def t_hemm(c, m, n, k, uplo=Uplo.Lower, side=Side.Left, **p):
    kk = m if side == Side.Left else n
    A = _herm_mat(c, kk, uplo, seed=1)
    B, C = c.mat(m, n, seed=2), c.mat(m, n, seed=3)
    Af, Bd, Cd = _herm_full(A), D(B), D(C)
    _, t = c.timed(lambda: sl.hemm(side, 1.0, A, B, 1.0, C, c.opts))
    ref = (Af @ Bd if side == Side.Left else Bd @ Af) + Cd
    err = _rel(D(C) - ref, Af.abs().max() * Bd.abs().max() * kk) if c.a.check == 'y' else None
    return err, t, 2.0 * m * n * kk


def t_trmm(c, m, n, k, side=Side.Left, uplo=Uplo.Lower, **p):
    kk = m if side == Side.Left else n
    T = c.mat(kk, kk, seed=1)
    Td = D(T)
    B = c.mat(m, n, seed=2)
    Bd = D(B)
    L = sl.TriangularMatrix(uplo, T)
    _, t = c.timed(lambda: sl.trmm(side, 1.0, L, B, c.opts))
    Tt = torch.tril(Td) if uplo == Uplo.Lower else torch.triu(Td)
    ref = Tt @ Bd if side == Side.Left else Bd @ Tt
    return (_rel(D(B) - ref, Td.abs().max() * Bd.abs().max() * kk) if c.a.check == 'y' else None), t, \
        1.0 * m * n * kk


def t_potrs(c, m, n, k, uplo=Uplo.Lower, **p):
    A = _herm_mat(c, n, uplo, "poev")
    Af = _herm_full(A)
    sl.potrf(A, c.opts)
    B = c.mat(n, k, seed=2)
    Bd = D(B)
    _, t = c.timed(lambda: sl.potrs(A, B, c.opts))
    err = _rel(Af @ D(B) - Bd, Af.abs().max() * D(B).abs().max() * n) if c.a.check == 'y' else None
    return err, t, 2.0 * n * n * k


def t_potri(c, m, n, k, uplo=Uplo.Lower, **p):
    A = _herm_mat(c, n, uplo, "poev")
    Af = _herm_full(A)
    def run():
        info = sl.potrf(A, c.opts)
        return info if info else sl.potri(A, c.opts)
    info, t = c.timed(run)
    err = _rel(_herm_full(A) @ Af - torch.eye(n, dtype=c.dt, device=Af.device), n) if c.a.check == 'y' else None
    return err if info == 0 else float("inf"), t, n ** 3


def t_trtri(c, m, n, k, uplo=Uplo.Lower, **p):
    T = c.mat(n, n, seed=1)
    Td = D(T) + n * torch.eye(n, dtype=c.dt, device=D(T).device)
    sl.from_dense(T, Td)
    L = sl.TriangularMatrix(uplo, T)
    info, t = c.timed(lambda: sl.trtri(L, c.opts))
    Tt = torch.tril(Td) if uplo == Uplo.Lower else torch.triu(Td)
    X = torch.tril(D(T)) if uplo == Uplo.Lower else torch.triu(D(T))
    err = _rel(X @ Tt - torch.eye(n, dtype=c.dt, device=Tt.device), n) if c.a.check == 'y' else None
    return err, t, n ** 3 / 3.0


def _lu_solve_check(c, A0, X, B0, n):
    return _rel(A0 @ X - B0, A0.abs().max() * X.abs().max() * n) if c.a.check == 'y' else None


def t_getrs(c, m, n, k, **p):
    A = c.mat(n, n, seed=1)
    Ad = D(A)
    piv = sl.Pivots()
    sl.getrf(A, piv, c.opts)
    B = c.mat(n, k, seed=2)
    Bd = D(B)
    _, t = c.timed(lambda: sl.getrs(A, piv, B, c.opts))
    return _lu_solve_check(c, Ad, D(B), Bd, n), t, 2.0 * n * n * k


def t_getri(c, m, n, k, **p):
    A = c.mat(n, n, seed=1)
    Ad = D(A)
    piv = sl.Pivots()
    def run():
        sl.getrf(A, piv, c.opts)
        return sl.getri(A, piv, c.opts)
    _, t = c.timed(run)
    err = _rel(D(A) @ Ad - torch.eye(n, dtype=c.dt, device=Ad.device), n * Ad.abs().max()) \
        if c.a.check == 'y' else None
    return err, t, 2.0 * n ** 3


def _getrf_method(method):
    def f(c, m, n, k, **p):
        from slate_amd.core.enums import MethodLU
        A, B = c.mat(n, n, "rand_dominant" if method == "nopiv" else "rands", 1), c.mat(n, k, seed=2)
        Ad, Bd = D(A), D(B)
        o = dict(c.opts)
        o[Option.MethodLU] = {"nopiv": MethodLU.NoPiv, "calu": MethodLU.CALU, "rbt": MethodLU.RBT}[method]
        _, t = c.timed(lambda: sl.gesv(A, sl.Pivots(), B, o))
        return _lu_solve_check(c, Ad, D(B), Bd, n), t, 2.0 * n ** 3 / 3.0
    return f


def t_posv_mixed(c, m, n, k, uplo=Uplo.Lower, **p):
    if c.t not in ('d', 'z'):
        return None, 0.0, 0.0
    A = _herm_mat(c, n, uplo, "poev")
    Af = _herm_full(A)
    B, X = c.mat(n, k, seed=2), c.mat(n, k, "zeros")
    Bd = D(B)
    _, t = c.timed(lambda: sl.posv_mixed(A, B, X, c.opts))
    return _lu_solve_check(c, Af, D(X), Bd, n), t, n ** 3 / 3.0


def t_gelqf(c, m, n, k, **p):
    A = c.mat(m, n, seed=1)
    Ad = D(A)
    T = sl.TriangularFactors()
    _, t = c.timed(lambda: sl.gelqf(A, T, c.opts))
    err = None
    if c.a.check == 'y':
        Q = c.mat(n, n, "identity", 1)
        sl.unmlq(Side.Left, Op.NoTrans, A, T, Q, c.opts)
        kk = min(m, n)
        err = _rel(torch.tril(D(A))[:, :kk] @ D(Q)[:kk] - Ad, Ad.abs().max() * n)
    return err, t, 2.0 * n * m * m - 2.0 * m ** 3 / 3.0


def t_cholqr(c, m, n, k, **p):
    A = c.mat(m, n, seed=1)
    Ad = D(A)
    R = c.mat(n, n, "zeros")
    info, t = c.timed(lambda: sl.cholqr(A, R, c.opts))
    err = _rel(D(A) @ torch.triu(D(R)) - Ad, Ad.abs().max() * m) if c.a.check == 'y' else None
    return err if info == 0 else float("inf"), t, 2.0 * m * n * n


def t_hegv(c, m, n, k, uplo=Uplo.Lower, **p):
    A = _herm_mat(c, n, uplo, seed=1)
    B = _herm_mat(c, n, uplo, "poev", seed=2)
    Af, Bf = _herm_full(A).cpu(), _herm_full(B).cpu()
    Z = c.mat(n, n, "zeros")
    w, t = c.timed(lambda: sl.hegv(1, A, B, None, Z, c.opts))
    X = D(Z).cpu()
    err = _rel(Af @ X - Bf @ X * w.cpu().to(c.dt), Af.abs().max() * Bf.abs().max() * n) \
        if c.a.check == 'y' else None
    return err, t, 14.0 * n ** 3 / 3.0


def t_gecondest(c, m, n, k, **p):
    A = c.mat(n, n, seed=1)
    Ad = D(A).cpu()
    anorm = float(sl.norm(Norm.One, A))
    piv = sl.Pivots()
    sl.getrf(A, piv, c.opts)
    r, t = c.timed(lambda: sl.gecondest(Norm.One, A, piv, anorm, c.opts))
    ref = 1.0 / (torch.linalg.norm(Ad, 1) * torch.linalg.norm(torch.linalg.inv(Ad), 1)).item()
    err = abs(r - ref) / ref if c.a.check == 'y' else None
    return (None if err is not None and err < 3.0 else err), t, 2.0 * n * n   # estimate within 3x


def t_colnorms(c, m, n, k, **p):
    A = c.mat(m, n, seed=1)
    Ad = D(A)
    v, t = c.timed(lambda: sl.colNorms(Norm.Max, A, c.opts))
    err = _rel(v.to(Ad.device).reshape(-1) - Ad.abs().max(0).values, Ad.abs().max()) if c.a.check == 'y' else None
    return err, t, 1.0 * m * n


def t_add(c, m, n, k, **p):
    A, B = c.mat(m, n, seed=1), c.mat(m, n, seed=2)
    Ad, Bd = D(A), D(B)
    _, t = c.timed(lambda: sl.add(2.0, A, -1.0, B, c.opts))
    return (_rel(D(B) - (2.0 * Ad - Bd), Ad.abs().max()) if c.a.check == 'y' else None), t, 2.0 * m * n


def t_redistribute(c, m, n, k, **p):
    A = c.mat(m, n, seed=1)
    B = sl.Matrix(m, n, nb=max(8, c.a.nb // 2 + 3), p=c.a.q, q=c.a.p, dtype=c.dt, device=c.dev)
    B.insertLocalTiles(device=c.dev.index if c.dev.type == "cuda" else -1)
    _, t = c.timed(lambda: sl.redistribute(A, B))
    return (_rel(D(B) - D(A), 1.0) if c.a.check == 'y' else None), t, 0.0


def t_gbsv(c, m, n, k, **p):
    kl = ku = max(1, c.a.nb // 2)
    A = sl.BandMatrix(n, n, kl, ku, nb=c.a.nb, p=c.a.p, q=c.a.q, dtype=c.dt, device=c.dev)
    A.insertLocalTiles(device=c.dev.index if c.dev.type == "cuda" else -1)
    sl.generate_matrix(A, "rand_dominant", 1)
    Ad = D(A)
    i = torch.arange(n, device=Ad.device)
    Ad = torch.where(((i[:, None] - i[None, :]) <= kl) & ((i[None, :] - i[:, None]) <= ku), Ad,
                     torch.zeros_like(Ad))                     # only the band is the operand
    B = c.mat(n, k, seed=2)
    Bd = D(B)
    info, t = c.timed(lambda: sl.gbsv(A, sl.Pivots(), B, c.opts))
    return _lu_solve_check(c, Ad, D(B), Bd, n), t, 2.0 * n * kl * (kl + ku)


def _band(c, n, kl, ku, seed=1):
    A = sl.BandMatrix(n, n, kl, ku, nb=c.a.nb, p=c.a.p, q=c.a.q, dtype=c.dt, device=c.dev)
    A.insertLocalTiles(device=c.dev.index if c.dev.type == "cuda" else -1)
    sl.generate_matrix(A, "rand_dominant", seed)
    sl.band_mask(A)
    return A


def t_pbsv(c, m, n, k, uplo=Uplo.Lower, **p):
    kd = max(1, c.a.nb // 2)
    A = sl.HermitianBandMatrix(uplo, n, kd, nb=c.a.nb, p=c.a.p, q=c.a.q, dtype=c.dt, device=c.dev)
    A.insertLocalTiles(device=c.dev.index if c.dev.type == "cuda" else -1)
    sl.generate_matrix(A, "poev", 1)
    sl.band_mask(A, kd, 0) if uplo == Uplo.Lower else sl.band_mask(A, 0, kd)
    Af = _herm_full(A)
    B = c.mat(n, k, seed=2)
    Bd = D(B)
    info, t = c.timed(lambda: sl.pbsv(A, B, c.opts))
    err = _rel(Af @ D(B) - Bd, Af.abs().max() * D(B).abs().max() * n) if c.a.check == 'y' else None
    return err, t, n * kd * kd + 4.0 * n * kd * k


def t_gbmm(c, m, n, k, **p):
    kl = ku = max(1, c.a.nb // 2)
    A = _band(c, n, kl, ku)
    B, C = c.mat(n, k, seed=2), c.mat(n, k, seed=3)
    Ad, Bd, Cd = D(A), D(B), D(C)
    _, t = c.timed(lambda: sl.gbmm(2.0, A, B, 0.5, C, c.opts))
    ref = 2.0 * Ad @ Bd + 0.5 * Cd
    err = _rel(D(C) - ref, ref.abs().max() * n) if c.a.check == 'y' else None
    return err, t, 2.0 * n * (kl + ku + 1) * k


def t_hbmm(c, m, n, k, uplo=Uplo.Lower, side=Side.Left, **p):
    kd = max(1, c.a.nb // 2)
    A = sl.HermitianBandMatrix(uplo, n, kd, nb=c.a.nb, p=c.a.p, q=c.a.q, dtype=c.dt, device=c.dev)
    A.insertLocalTiles(device=c.dev.index if c.dev.type == "cuda" else -1)
    sl.generate_matrix(A, "rands_hermitian", 1)
    sl.band_mask(A, kd, 0) if uplo == Uplo.Lower else sl.band_mask(A, 0, kd)
    Af = _herm_full(A)
    B = c.mat(n, k, seed=2) if side == Side.Left else c.mat(k, n, seed=2)
    C = c.mat(n, k, "zeros") if side == Side.Left else c.mat(k, n, "zeros")
    Bd = D(B)
    _, t = c.timed(lambda: sl.hbmm(side, 1.0, A, B, 0.0, C, c.opts))
    ref = Af @ Bd if side == Side.Left else Bd @ Af
    err = _rel(D(C) - ref, ref.abs().max() * n) if c.a.check == 'y' else None
    return err, t, 2.0 * n * (2 * kd + 1) * k


def t_tbsm(c, m, n, k, uplo=Uplo.Lower, side=Side.Left, **p):
    kd = max(1, c.a.nb // 2)
    T = sl.TriangularBandMatrix(uplo, Diag.NonUnit, n, kd, nb=c.a.nb, p=c.a.p, q=c.a.q, dtype=c.dt, device=c.dev)
    T.insertLocalTiles(device=c.dev.index if c.dev.type == "cuda" else -1)
    sl.generate_matrix(T, "rand_dominant", 1)
    sl.band_mask(T, kd, 0) if uplo == Uplo.Lower else sl.band_mask(T, 0, kd)
    Td = D(T)
    B = c.mat(n, k, seed=2) if side == Side.Left else c.mat(k, n, seed=2)
    Bd = D(B)
    _, t = c.timed(lambda: sl.tbsm(side, 1.0, T, B, None, c.opts))
    X = D(B)
    ref = Td @ X if side == Side.Left else X @ Td
    err = _rel(ref - Bd, Td.abs().max() * X.abs().max() * n) if c.a.check == 'y' else None
    return err, t, 1.0 * n * kd * k * 2


def t_pocondest(c, m, n, k, uplo=Uplo.Lower, **p):
    A = _herm_mat(c, n, uplo, "poev")
    Af = _herm_full(A)
    anorm = sl.norm(Norm.One, A)
    sl.potrf(A, c.opts)
    rc, t = c.timed(lambda: sl.pocondest(Norm.One, A, anorm, c.opts))
    ref = 1.0 / float(torch.linalg.cond(Af.cpu(), 1))
    return (0.0 if ref / 3 <= rc <= 3 * ref else 1.0) if c.a.check == 'y' else None, t, 4.0 * n * n


def t_trcondest(c, m, n, k, uplo=Uplo.Lower, **p):
    A = c.mat(n, n, "rand_dominant", 1)
    T = sl.TriangularMatrix(uplo, A, diag=Diag.NonUnit)
    Td = torch.tril(D(A)) if uplo == Uplo.Lower else torch.triu(D(A))
    rc, t = c.timed(lambda: sl.trcondest(Norm.One, T, None, c.opts))
    ref = 1.0 / float(torch.linalg.cond(Td.cpu(), 1))
    return (0.0 if ref / 3 <= rc <= 3 * ref else 1.0) if c.a.check == 'y' else None, t, 4.0 * n * n


def t_unmqr(c, m, n, k, side=Side.Left, **p):
    A = c.mat(m, n, seed=1)
    T = sl.TriangularFactors()
    sl.geqrf(A, T, c.opts)
    C = c.mat(m, k, seed=2) if side == Side.Left else c.mat(k, m, seed=2)
    Cd = D(C)
    _, t = c.timed(lambda: sl.unmqr(side, Op.ConjTrans, A, T, C, c.opts))
    sl.unmqr(side, Op.NoTrans, A, T, C, c.opts)                     # Q Q^H C = C
    err = _rel(D(C) - Cd, Cd.abs().max() * m) if c.a.check == 'y' else None
    return err, t, 4.0 * m * n * k


def t_gesv_mixed_gmres(c, m, n, k, **p):
    if c.t not in ('d', 'z'):
        return None, 0.0, 0.0
    A, B = c.mat(n, n, "rand_dominant", 1), c.mat(n, k, seed=2)
    X = c.mat(n, k, "zeros")
    Ad, Bd = D(A), D(B)
    r, t = c.timed(lambda: sl.gesv_mixed_gmres(A, sl.Pivots(), B, X, c.opts))
    err = _rel(Ad @ D(X) - Bd, Ad.abs().max() * D(X).abs().max() * n) if c.a.check == 'y' else None
    return err, t, 2.0 * n ** 3 / 3.0


def t_svd_vals(c, m, n, k, **p):
    A = c.mat(m, n, "svd_geo", 1)
    s0 = torch.linalg.svdvals(D(A).cpu())
    s, t = c.timed(lambda: sl.svd_vals(A, None, c.opts))
    err = _rel(s.cpu() - s0, s0.max() * max(m, n)) if c.a.check == 'y' else None
    return err, t, 4.0 * m * n * n


def t_heev_vals(c, m, n, k, uplo=Uplo.Lower, **p):
    A = c.mat(n, n, "heev_arith", 1, sl.HermitianMatrix, uplo=uplo)
    w0 = torch.linalg.eigvalsh(_herm_full(A).cpu())
    w, t = c.timed(lambda: sl.heev(A, None, None, c.opts))
    err = _rel(w.cpu() - w0, w0.abs().max() * n) if c.a.check == 'y' else None
    return err, t, 4.0 * n ** 3 / 3.0


def t_matgen(c, m, n, k, **p):
    """Generation rate of the spectral svd kind (two distributed QRs)."""
    A = c.mat(m, n, "zeros")
    s, t = c.timed(lambda: sl.generate_matrix(A, "svd_geo", 1, cond=1e3))
    err = _rel(torch.linalg.svdvals(D(A).cpu()) - s.sort(descending=True).values, 1.0) if c.a.check == 'y' else None
    return err, t, 8.0 * m * n * n


# ------------------------------------------------------- aux by structure
def _struct(c, kind, m, n, uplo, seed):
    """A general matrix of the tester's grid viewed as `kind`: ge | tz | tr |
    he | sy (test/test_add.cc, test_copy.cc, test_scale.cc, test_set.cc,
    test_norm.cc sweep the same five)."""
    if kind in ("tr", "he", "sy"):
        m = n
    M = c.mat(m, n, seed=seed)
    if kind == "ge":
        return M, torch.ones(m, n, dtype=torch.bool)
    i = torch.arange(m)[:, None]
    j = torch.arange(n)[None, :]
    mask = (i >= j) if uplo == Uplo.Lower else (i <= j)
    if kind == "tz":
        return sl.TrapezoidMatrix(uplo, matrix=M), mask
    if kind == "tr":
        return sl.TriangularMatrix(uplo, M), mask
    return (sl.HermitianMatrix if kind == "he" else sl.SymmetricMatrix)(uplo, M), mask


def _full_of(kind, Dm, mask):
    """The operand the structure represents (Hermitian/symmetric: both
    triangles from the stored one)."""
    if kind in ("he", "sy"):
        L = torch.where(mask.to(Dm.device), Dm, torch.zeros_like(Dm))
        R = L.mH if kind == "he" else L.mT
        F = L + R
        F.diagonal().copy_(Dm.diagonal().real.to(Dm.dtype) if kind == "he" else Dm.diagonal())
        return F
    return torch.where(mask.to(Dm.device), Dm, torch.zeros_like(Dm))


def _aux(kind, op):
    def f(c, m, n, k, uplo=Uplo.Lower, **p):
        A, mask = _struct(c, kind, m, n, uplo, 1)
        Ad = D(A).clone()
        mk = mask.to(Ad.device)
        mm, nn = Ad.shape
        chk = c.a.check == 'y'
        if op == "norm":
            v, t = c.timed(lambda: sl.norm(Norm.Fro, A, c.opts))
            ref = torch.linalg.norm(_full_of(kind, Ad, mask))
            return (abs(float(v) - float(ref)) / max(float(ref), 1e-300) if chk else None), t, 2.0 * mm * nn
        if op in ("add", "copy"):
            B, _ = _struct(c, kind, m, n, uplo, 2)
            Bd = D(B).clone()
            if op == "add":
                _, t = c.timed(lambda: sl.add(2.0, A, -1.0, B, c.opts))
                ref = torch.where(mk, 2.0 * Ad - Bd, Bd)
            else:
                _, t = c.timed(lambda: sl.copy(A, B, c.opts))
                ref = torch.where(mk, Ad, Bd)
            got = D(B)
            return (_rel(torch.where(mk, got - ref, torch.zeros_like(got)), Ad.abs().max() + Bd.abs().max())
                    if chk else None), t, 2.0 * mm * nn
        if op == "scale":
            _, t = c.timed(lambda: sl.scale(3.0, 2.0, A, c.opts))
            ref = torch.where(mk, Ad * 1.5, Ad)
        else:                                              # set
            _, t = c.timed(lambda: sl.set(0.5, 2.0, A, c.opts))
            i = torch.arange(mm, device=Ad.device)[:, None]
            j = torch.arange(nn, device=Ad.device)[None, :]
            val = torch.where(i == j, torch.full_like(Ad, 2.0), torch.full_like(Ad, 0.5))
            ref = torch.where(mk, val, Ad)
        got = D(A)
        return (_rel(torch.where(mk, got - ref, torch.zeros_like(got)), Ad.abs().max() + 2.0) if chk else None), \
            t, 1.0 * mm * nn
    return f


def t_scale_row_col(c, m, n, k, **p):
    A = c.mat(m, n, seed=1)
    Ad = D(A)
    R = torch.rand(m, dtype=torch.float64, generator=torch.Generator().manual_seed(3)) + 0.5
    Cc = torch.rand(n, dtype=torch.float64, generator=torch.Generator().manual_seed(4)) + 0.5
    from slate_amd.core.enums import Equed
    _, t = c.timed(lambda: sl.scale_row_col(Equed.Both, R, Cc, A, c.opts))
    ref = Ad * R.to(Ad.device, c.dt)[:, None] * Cc.to(Ad.device, c.dt)[None, :]
    return (_rel(D(A) - ref, Ad.abs().max() * 2.25) if c.a.check == 'y' else None), t, 2.0 * m * n


def t_bandnorm(herm):
    def f(c, m, n, k, uplo=Uplo.Lower, **p):
        kd = max(1, c.a.nb // 2)
        if herm:
            A = sl.HermitianBandMatrix(uplo, n, kd, nb=c.a.nb, p=c.a.p, q=c.a.q, dtype=c.dt, device=c.dev)
        else:
            A = sl.BandMatrix(n, n, kd, kd, nb=c.a.nb, p=c.a.p, q=c.a.q, dtype=c.dt, device=c.dev)
        A.insertLocalTiles(device=c.dev.index if c.dev.type == "cuda" else -1)
        sl.generate_matrix(A, "rands", 1)
        if herm:
            sl.band_mask(A, kd, 0) if uplo == Uplo.Lower else sl.band_mask(A, 0, kd)
            F = _herm_full(A)
        else:
            sl.band_mask(A)
            F = D(A)
        v, t = c.timed(lambda: (sl.hbnorm if herm else sl.gbnorm)(Norm.One, A, c.opts))
        ref = torch.linalg.matrix_norm(F, 1)
        return (abs(float(v) - float(ref)) / float(ref) if c.a.check == 'y' else None), t, 2.0 * n * kd
    return f


# ----------------------------------------------------- factor/solve pieces
def t_getrf_variant(method):
    def f(c, m, n, k, **p):
        A = c.mat(n, n, "rand_dominant" if method == "nopiv" else "rands", 1)
        Ad = D(A)
        piv = sl.Pivots()
        fn = {"nopiv": lambda: sl.getrf_nopiv(A, c.opts), "tntpiv": lambda: sl.getrf_tntpiv(A, piv, c.opts)}[method]
        _, t = c.timed(fn)
        if c.a.check != 'y':
            return None, t, 2.0 * n ** 3 / 3.0
        F = D(A)
        L = torch.tril(F, -1) + torch.eye(n, dtype=c.dt, device=F.device)
        PA = Ad.clone()
        if method != "nopiv":
            for i, pv in enumerate(piv.ipiv.tolist()):
                if pv != i:
                    PA[[i, pv]] = PA[[pv, i]]
        return _rel(L @ torch.triu(F) - PA, Ad.abs().max() * n), t, 2.0 * n ** 3 / 3.0
    return f


def t_getrs_variant(method):
    def f(c, m, n, k, **p):
        A = c.mat(n, n, "rand_dominant" if method == "nopiv" else "rands", 1)
        Ad = D(A)
        piv = sl.Pivots()
        if method == "nopiv":
            sl.getrf_nopiv(A, c.opts)
        else:
            sl.getrf_tntpiv(A, piv, c.opts)
        B = c.mat(n, k, seed=2)
        Bd = D(B)
        run = (lambda: sl.getrs_nopiv(A, B, c.opts)) if method == "nopiv" else (lambda: sl.getrs_tntpiv(A, piv, B, c.opts))
        _, t = c.timed(run)
        return _lu_solve_check(c, Ad, D(B), Bd, n), t, 2.0 * n * n * k
    return f


def t_gbtrf_gbtrs(solve):
    def f(c, m, n, k, **p):
        kl = ku = max(1, c.a.nb // 2)
        A = _band(c, n, kl, ku)
        Ad = D(A)
        piv = sl.Pivots()
        if not solve:
            info, t = c.timed(lambda: sl.gbtrf(A, piv, c.opts))
            B = c.mat(n, 1, seed=2)
            Bd = D(B)
            sl.gbtrs(A, piv, B, c.opts)
            return _lu_solve_check(c, Ad, D(B), Bd, n), t, 2.0 * n * kl * (kl + ku)
        sl.gbtrf(A, piv, c.opts)
        B = c.mat(n, k, seed=2)
        Bd = D(B)
        _, t = c.timed(lambda: sl.gbtrs(A, piv, B, c.opts))
        return _lu_solve_check(c, Ad, D(B), Bd, n), t, 2.0 * n * (2 * kl + ku) * k
    return f


def t_pbtrf_pbtrs(solve):
    def f(c, m, n, k, uplo=Uplo.Lower, **p):
        kd = max(1, c.a.nb // 2)
        A = sl.HermitianBandMatrix(uplo, n, kd, nb=c.a.nb, p=c.a.p, q=c.a.q, dtype=c.dt, device=c.dev)
        A.insertLocalTiles(device=c.dev.index if c.dev.type == "cuda" else -1)
        sl.generate_matrix(A, "poev", 1)
        sl.band_mask(A, kd, 0) if uplo == Uplo.Lower else sl.band_mask(A, 0, kd)
        Af = _herm_full(A)
        B = c.mat(n, k, seed=2)
        Bd = D(B)
        if solve:
            sl.pbtrf(A, c.opts)
            _, t = c.timed(lambda: sl.pbtrs(A, B, c.opts))
        else:
            _, t = c.timed(lambda: sl.pbtrf(A, c.opts))
            sl.pbtrs(A, B, c.opts)
        err = _rel(Af @ D(B) - Bd, Af.abs().max() * D(B).abs().max() * n) if c.a.check == 'y' else None
        return err, t, (4.0 * n * kd * k) if solve else (n * kd * kd)
    return f


def t_hetrf_hetrs(solve):
    def f(c, m, n, k, **p):
        A, B = c.mat(n, n, seed=1, cls=sl.HermitianMatrix), c.mat(n, k, seed=2)
        Af, Bd = _herm_full(A), D(B)
        piv = sl.Pivots()
        if solve:
            sl.hetrf(A, piv, None, None, None, c.opts)
            _, t = c.timed(lambda: sl.hetrs(A, piv, None, None, B, c.opts))
        else:
            _, t = c.timed(lambda: sl.hetrf(A, piv, None, None, None, c.opts))
            sl.hetrs(A, piv, None, None, B, c.opts)
        err = _rel(Af @ D(B) - Bd, Af.abs().max() * D(B).abs().max() * n) if c.a.check == 'y' else None
        return err, t, (2.0 * n * n * k) if solve else (n ** 3 / 3.0)
    return f


def t_posv_mixed_gmres(c, m, n, k, uplo=Uplo.Lower, **p):
    if c.t not in ('d', 'z'):
        return None, 0.0, 0.0
    A = _herm_mat(c, n, uplo, "poev")
    Af = _herm_full(A)
    B, X = c.mat(n, 1, seed=2), c.mat(n, 1, "zeros")
    Bd = D(B)
    _, t = c.timed(lambda: sl.posv_mixed_gmres(A, B, X, c.opts))
    return _lu_solve_check(c, Af, D(X), Bd, n), t, n ** 3 / 3.0


def t_hegst(c, m, n, k, uplo=Uplo.Lower, **p):
    A = _herm_mat(c, n, uplo, seed=1)
    B = _herm_mat(c, n, uplo, "poev", seed=2)
    Af, Bf = _herm_full(A), _herm_full(B)
    sl.potrf(B, c.opts)
    _, t = c.timed(lambda: sl.hegst(1, A, B, c.opts))
    if c.a.check != 'y':
        return None, t, n ** 3
    Fb = D(B)
    L = torch.tril(Fb) if uplo == Uplo.Lower else torch.triu(Fb).mH
    # itype 1: C = L^{-1} A L^{-H}; check L C L^H = A
    C = _herm_full(A)
    return _rel(L @ C @ L.mH - Af, Af.abs().max() * n), t, 1.0 * n ** 3


# ------------------------------------------------ two-stage eig / SVD stages
def _dense_cm(c, m, n, seed, herm=False):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(m, n, dtype=c.dt, generator=g)
    if herm:
        X = X + X.mH
    return X.to(c.dev).t().contiguous().t()


def t_he2hb(c, m, n, k, **p):
    from slate_amd.models import eig as E
    nb = max(2, min(c.a.nb, 64))
    A0 = _dense_cm(c, n, n, 1, herm=True)
    Af = A0.clone()
    F, t = c.timed(lambda: sl.he2hb(Af, nb))
    if c.a.check != 'y':
        return None, t, 4.0 * n ** 3 / 3.0
    band = E._band_only(Af, nb)
    w0, w1 = torch.linalg.eigvalsh(A0.cpu()), torch.linalg.eigvalsh(band.cpu())
    return _rel(w1 - w0, w0.abs().max() * n), t, 4.0 * n ** 3 / 3.0


def _band_herm(c, n, b, seed=1):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, n, dtype=c.dt, generator=g)
    X = X + X.mH
    i = torch.arange(n)
    X = torch.where((i[:, None] - i[None, :]).abs() <= b, X, torch.zeros_like(X))
    return X.to(c.dev).t().contiguous().t()


def t_hb2st(c, m, n, k, **p):
    b = max(1, min(c.a.nb, 64))
    B0 = _band_herm(c, n, b)
    (d, e, F), t = c.timed(lambda: sl.hb2st(B0.clone(), b, device=c.dev if c.dev.type == "cuda" else None))
    if c.a.check != 'y':
        return None, t, 6.0 * n * n * b
    w0 = torch.linalg.eigvalsh(B0.cpu())
    w1 = torch.linalg.eigvalsh(torch.diag(d) + torch.diag(e, 1) + torch.diag(e, -1))
    return _rel(w1 - w0, w0.abs().max() * n), t, 6.0 * n * n * b


def t_unmtr_hb2st(c, m, n, k, **p):
    b = max(1, min(c.a.nb, 64))
    B0 = _band_herm(c, n, b)
    d, e, F = sl.hb2st(B0.clone(), b, device=c.dev if c.dev.type == "cuda" else None)
    w, Zt = sl.stedc(d, e, device=c.dev)
    Z = Zt.to(c.dt).to(c.dev).t().contiguous().t()
    _, t = c.timed(lambda: sl.unmtr_hb2st(F, Z))
    err = _rel(B0 @ Z - Z * w.to(c.dev, c.dt), B0.abs().max() * n) if c.a.check == 'y' else None
    return err, t, 2.0 * n * n * b


def t_unmtr_he2hb(c, m, n, k, **p):
    from slate_amd.models import eig as E
    nb = max(2, min(c.a.nb, 64))
    A0 = _dense_cm(c, n, n, 1, herm=True)
    Af = A0.clone()
    F = sl.he2hb(Af, nb)
    band = E._band_only(Af, nb)
    w, V = torch.linalg.eigh(band.cpu())
    Z = V.to(c.dev).t().contiguous().t()
    _, t = c.timed(lambda: sl.unmtr_he2hb(F, Z))
    err = _rel(A0 @ Z - Z * w.to(c.dev, c.dt), A0.abs().max() * n) if c.a.check == 'y' else None
    return err, t, 2.0 * n ** 3


def _tridiag(n, seed=1):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, dtype=torch.float64, generator=g), torch.randn(max(n - 1, 0), dtype=torch.float64, generator=g)


def _trid_check(c, d, e, w, Z=None):
    T = torch.diag(d) + torch.diag(e, 1) + torch.diag(e, -1)
    w0 = torch.linalg.eigvalsh(T)
    sc = w0.abs().max() * d.numel()
    err = _rel(w.cpu() - w0, sc)
    if Z is not None:
        Zc = Z.cpu().to(torch.float64)
        err = max(err, _rel(T @ Zc - Zc * w.cpu(), sc))
    return err


def t_sterf(c, m, n, k, **p):
    d, e = _tridiag(n)
    w, t = c.timed(lambda: sl.sterf(d, e))
    return (_trid_check(c, d, e, w) if c.a.check == 'y' else None), t, 30.0 * n * n


def t_steqr(c, m, n, k, **p):
    d, e = _tridiag(n)
    (w, Z), t = c.timed(lambda: sl.steqr(d, e))
    return (_trid_check(c, d, e, w, Z) if c.a.check == 'y' else None), t, 6.0 * n ** 3


def t_stedc(c, m, n, k, **p):
    d, e = _tridiag(n)
    (w, Z), t = c.timed(lambda: sl.stedc(d, e, device=c.dev))
    return (_trid_check(c, d, e, w, Z) if c.a.check == 'y' else None), t, 4.0 * n ** 3 / 3.0


def _secular_problem(n, seed=1):
    g = torch.Generator().manual_seed(seed)
    dd = torch.sort(torch.randn(n, dtype=torch.float64, generator=g)).values
    z = torch.randn(n, dtype=torch.float64, generator=g)
    return dd, z / z.norm(), 0.75


def t_stedc_sort(c, m, n, k, **p):
    g = torch.Generator().manual_seed(2)
    dd = torch.randn(n, dtype=torch.float64, generator=g)
    z = torch.randn(n, dtype=torch.float64, generator=g)
    Q = torch.eye(n, dtype=torch.float64)
    (ds, zs, Qs), t = c.timed(lambda: sl.stedc_sort(dd, z, Q))
    ok = bool((ds[1:] >= ds[:-1]).all()) and torch.allclose(Qs.T @ dd, ds) and torch.allclose(Qs.T @ z, zs)
    return (0.0 if ok else 1.0) if c.a.check == 'y' else None, t, 0.0


def t_stedc_deflate(c, m, n, k, **p):
    dd, z, rho = _secular_problem(n)
    dd[1::4] = dd[0::4][:dd[1::4].numel()]              # repeated poles
    dd = torch.sort(dd).values
    z[2::5] = 0.0                                         # zero weights
    Q = torch.eye(n, dtype=torch.float64)
    M0 = torch.diag(dd) + rho * torch.outer(z, z)
    (z2, K), t = c.timed(lambda: sl.stedc_deflate(dd, z.clone(), rho, Q))
    # the deflated problem is similar to the original: Q^T M0 Q = diag(dd) + rho z2 z2^T
    M1 = torch.diag(dd) + rho * torch.outer(z2, z2)
    err = _rel(Q.T @ M0 @ Q - M1, M0.abs().max() * n) if c.a.check == 'y' else None
    return err, t, 0.0


def t_stedc_secular(c, m, n, k, **p):
    dd, z, rho = _secular_problem(n)
    (lam, org, mu), t = c.timed(lambda: sl.stedc_secular(dd, z, rho))
    w0 = torch.linalg.eigvalsh(torch.diag(dd) + rho * torch.outer(z, z))
    return (_rel(torch.sort(lam).values - w0, w0.abs().max() * n) if c.a.check == 'y' else None), t, 20.0 * n * n


def t_stedc_z_vector(c, m, n, k, **p):
    dd, z, rho = _secular_problem(n)
    lam, org, mu = sl.stedc_secular(dd, z, rho)
    (zh, V), t = c.timed(lambda: sl.stedc_z_vector(dd, z, rho, org, mu))
    M = torch.diag(dd) + rho * torch.outer(z, z)
    err = _rel(M @ V - V * lam, M.abs().max() * n) if c.a.check == 'y' else None
    return err, t, 3.0 * n * n


def t_ge2tb(c, m, n, k, **p):
    nb = max(2, min(c.a.nb, 64))
    mm = max(m, n)
    A0 = _dense_cm(c, mm, n, 1)
    Af = A0.clone()
    F, t = c.timed(lambda: sl.ge2tb(Af, nb))
    if c.a.check != 'y':
        return None, t, 4.0 * mm * n * n
    i = torch.arange(n, device=Af.device)
    dl = i[None, :] - i[:, None]
    band = torch.where((dl >= 0) & (dl <= nb), Af[:n], torch.zeros_like(Af[:n]))
    s0, s1 = torch.linalg.svdvals(A0.cpu()), torch.linalg.svdvals(band.cpu())
    return _rel(s1 - s0, s0.max() * mm), t, 4.0 * mm * n * n


def _band_upper(c, n, b, seed=1):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, n, dtype=c.dt, generator=g)
    i = torch.arange(n)
    dl = i[None, :] - i[:, None]
    X = torch.where((dl >= 0) & (dl <= b), X, torch.zeros_like(X))
    return X.to(c.dev).t().contiguous().t()


def t_tb2bd(c, m, n, k, **p):
    b = max(1, min(c.a.nb, 64))
    B0 = _band_upper(c, n, b)
    (d, e, F), t = c.timed(lambda: sl.tb2bd(B0.clone(), b))
    if c.a.check != 'y':
        return None, t, 8.0 * n * n * b
    s0 = torch.linalg.svdvals(B0.cpu())
    s1 = torch.linalg.svdvals(torch.diag(d) + torch.diag(e, 1))
    return _rel(s1 - s0, s0.max() * n), t, 8.0 * n * n * b


def t_unmbr_tb2bd(c, m, n, k, **p):
    b = max(1, min(c.a.nb, 64))
    B0 = _band_upper(c, n, b)
    d, e, F = sl.tb2bd(B0.clone(), b)
    Bd = (torch.diag(d) + torch.diag(e, 1)).to(c.dt)
    ZU = torch.eye(n, dtype=c.dt, device=c.dev).t()
    ZV = torch.eye(n, dtype=c.dt, device=c.dev).t()
    _, t = c.timed(lambda: (sl.unmbr_tb2bd('L', F, ZU), sl.unmbr_tb2bd('R', F, ZV)))
    err = _rel(ZU.cpu() @ Bd @ ZV.cpu().mH - B0.cpu(), B0.abs().max() * n) if c.a.check == 'y' else None
    return err, t, 4.0 * n * n * b


def t_bdsqr(c, m, n, k, **p):
    d, e = _tridiag(n)
    (s, U, VT), t = c.timed(lambda: sl.bdsqr(d, e))
    if c.a.check != 'y':
        return None, t, 12.0 * n ** 3
    B = torch.diag(d) + torch.diag(e, 1)
    s0 = torch.linalg.svdvals(B)
    err = max(_rel(torch.sort(s, descending=True).values - s0, s0.max() * n),
              _rel(U @ torch.diag(s) @ VT - B, s0.max() * n))
    return err, t, 12.0 * n ** 3


ROUTINES = {"gemm": t_gemm, "herk": t_herk, "syrk": t_herk, "trsm": t_trsm, "potrf": t_potrf,
            "posv": t_posv, "getrf": t_getrf, "gesv": t_gesv, "geqrf": t_geqrf, "gels": t_gels,
            "heev": t_heev, "syev": t_heev, "svd": t_svd, "norm": t_norm, "genorm": t_norm,
            "gesv_mixed": t_gesv_mixed, "hesv": t_hesv, "sysv": t_hesv,
            "her2k": t_her2k, "syr2k": t_her2k, "hemm": t_hemm, "symm": t_hemm, "trmm": t_trmm,
            "potrs": t_potrs, "potri": t_potri, "trtri": t_trtri, "getrs": t_getrs, "getri": t_getri,
            "gesv_nopiv": _getrf_method("nopiv"), "gesv_tntpiv": _getrf_method("calu"),
            "gesv_calu": _getrf_method("calu"), "gesv_rbt": _getrf_method("rbt"),
            "posv_mixed": t_posv_mixed, "gelqf": t_gelqf, "cholqr": t_cholqr, "hegv": t_hegv,
            "sygv": t_hegv, "gecondest": t_gecondest, "colnorms": t_colnorms, "add": t_add,
            "redistribute": t_redistribute, "gbsv": t_gbsv, "pbsv": t_pbsv, "gbmm": t_gbmm, "hbmm": t_hbmm,
            "tbsm": t_tbsm, "pocondest": t_pocondest, "trcondest": t_trcondest, "unmqr": t_unmqr,
            "gesv_mixed_gmres": t_gesv_mixed_gmres, "svd_vals": t_svd_vals, "heev_vals": t_heev_vals,
            "syev_vals": t_heev_vals, "matgen": t_matgen,
            "scale_row_col": t_scale_row_col, "gbnorm": t_bandnorm(False), "hbnorm": t_bandnorm(True),
            "getrf_nopiv": t_getrf_variant("nopiv"), "getrf_tntpiv": t_getrf_variant("tntpiv"),
            "getrs_nopiv": t_getrs_variant("nopiv"), "getrs_tntpiv": t_getrs_variant("tntpiv"),
            "gbtrf": t_gbtrf_gbtrs(False), "gbtrs": t_gbtrf_gbtrs(True), "pbtrf": t_pbtrf_pbtrs(False),
            "pbtrs": t_pbtrf_pbtrs(True), "hetrf": t_hetrf_hetrs(False), "hetrs": t_hetrf_hetrs(True),
            "sytrf": t_hetrf_hetrs(False), "sytrs": t_hetrf_hetrs(True), "posv_mixed_gmres": t_posv_mixed_gmres,
            "hegst": t_hegst, "he2hb": t_he2hb, "hb2st": t_hb2st, "unmtr_hb2st": t_unmtr_hb2st,
            "unmtr_he2hb": t_unmtr_he2hb, "sterf": t_sterf, "steqr": t_steqr, "stedc": t_stedc,
            "stedc_sort": t_stedc_sort, "stedc_deflate": t_stedc_deflate, "stedc_secular": t_stedc_secular,
            "stedc_z_vector": t_stedc_z_vector, "ge2tb": t_ge2tb, "tb2bd": t_tb2bd, "unmbr_tb2bd": t_unmbr_tb2bd,
            "bdsqr": t_bdsqr}
for _k, _pfx in (("ge", ""), ("tz", "tz"), ("tr", "tr"), ("he", "he"), ("sy", "sy")):
    for _op in ("add", "copy", "scale", "set", "norm"):
        if _k == "ge" and _op in ("add", "norm"):
            continue                                   # generic add / genorm above
        ROUTINES[(_pfx or "") + _op] = _aux(_k, _op)

# per-GPU dense peaks (MI355X spec, TFLOP/s): fp64 matrix = vector, fp32 matrix
PEAK_TF = {'s': 157.3, 'd': 78.6, 'c': 157.3, 'z': 78.6}


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
              f"{'time(s)':>9} {'Gflop/s':>9} {'%peak':>6}  status", flush=True)
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
                # complex flops count 4 real ones (LAPACK++ Gflop<complex>)
                gfr = gf * (4 if t in ('c', 'z') else 1)
                pk = f"{100 * gfr / (1e3 * PEAK_TF[t] * comm.size):6.1f}" if ctx.dev.type == "cuda" else f"{'-':>6}"
                print(f"{t:>4} {m:>6} {n:>6} {k:>6} {a.nb:>5} {f'{a.p}x{a.q}':>6} {up:>4} {es:>10} {tm:9.4f} "
                      f"{gf:9.1f} {pk}  {'pass' if ok else 'FAILED'}", flush=True)
    if comm.rank == 0:
        print("All tests passed." if fails == 0 else f"{fails} tests FAILED.", flush=True)
    sl.finalize()
    return 1 if fails else 0


if __name__ == "__main__":
    sys.exit(main())
