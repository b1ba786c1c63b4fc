"""Distributed drivers on CPU: single rank and gloo grids 2x1, 1x2, 2x2.

Reference test strategy (test/test_*.cc): run the routine on a random
matrix, compare against a sequential reference (here PyTorch fp64 on the
gathered matrix), residual-based tolerances.
"""
import pytest
import torch

import slate_amd as sl
from slate_amd.core.enums import Diag, Norm, Op, Side, Uplo
from slate_amd.models.aux import allgather_dense as D

from dist_util import run_dist


def mat(m, n, nb, seed, p=1, q=1, dt=torch.float64, kind="rands"):
    A = sl.Matrix(m, n, nb=nb, p=p, q=q, dtype=dt)
    A.insertLocalTiles()
    sl.generate_matrix(A, kind, seed)
    return A


def herm(n, nb, seed, p=1, q=1, dt=torch.float64, uplo=Uplo.Lower):
    A = sl.HermitianMatrix(uplo, n, nb=nb, p=p, q=q, dtype=dt)
    A.insertLocalTiles()
    sl.generate_matrix(A, "poev", seed)
    return A


def full_herm(A):
    X = D(A)
    L = torch.tril(X) if A.uploPhysical() == Uplo.Lower else torch.triu(X)
    return L + L.mH - torch.diag(torch.diagonal(L))


def close(a, b, tol=1e-10):
    s = max(1.0, b.abs().max().item())
    err = (a - b).abs().max().item() / s
    assert err < tol, err


# ----------------------------------------------------------------- checks
def check_gemm(p, q, dt=torch.float64):
    for ta, tb in [(Op.NoTrans, Op.NoTrans), (Op.ConjTrans, Op.NoTrans), (Op.NoTrans, Op.Trans)]:
        A = mat(70, 50, 16, 1, p, q, dt) if ta == Op.NoTrans else mat(50, 70, 16, 1, p, q, dt)
        B = mat(50, 40, 16, 2, p, q, dt) if tb == Op.NoTrans else mat(40, 50, 16, 2, p, q, dt)
        C = mat(70, 40, 16, 3, p, q, dt)
        Ad, Bd, Cd = D(A), D(B), D(C)
        opA = A if ta == Op.NoTrans else A.conj_transpose()
        opB = B if tb == Op.NoTrans else B.transpose()
        sl.gemm(1.5, opA, opB, -0.5, C)
        ref = 1.5 * (Ad if ta == Op.NoTrans else Ad.mH) @ (Bd if tb == Op.NoTrans else Bd.T) - 0.5 * Cd
        close(D(C), ref)


def check_herk_trsm_trmm(p, q, dt=torch.float64):
    A = mat(60, 30, 16, 4, p, q, dt)
    C = herm(60, 16, 5, p, q, dt)
    Cf = full_herm(C)
    Ad = D(A)
    sl.herk(2.0, A, 0.5, C)
    close(full_herm(C), 2.0 * Ad @ Ad.mH + 0.5 * Cf)
    # trsm / trmm, left lower and right upper
    T = mat(48, 48, 16, 6, p, q, dt)
    sl.add(0.0, T, 1.0, T)
    Td = D(T) + 48 * torch.eye(48, dtype=dt)
    sl.from_dense(T, Td)
    B = mat(48, 20, 16, 7, p, q, dt)
    Bd = D(B)
    L = sl.TriangularMatrix(Uplo.Lower, T, diag=Diag.NonUnit)
    sl.trsm(Side.Left, 2.0, L, B)
    close(D(B), torch.linalg.solve_triangular(torch.tril(Td), 2.0 * Bd, upper=False), 1e-9)
    B2 = mat(20, 48, 16, 8, p, q, dt)
    B2d = D(B2)
    U = sl.TriangularMatrix(Uplo.Upper, T, diag=Diag.NonUnit)
    sl.trmm(Side.Right, 1.0, U, B2)
    close(D(B2), B2d @ torch.triu(Td))


def check_potrf(p, q, dt=torch.float64, uplo=Uplo.Lower):
    # n = 100: an odd tile count with a ragged last tile (the unpaired last
    # step of the step-pair trailing update, chol.py)
    for n in (100, 96):
        nb = 16
        A = herm(n, nb, 11, p, q, dt, uplo)
        Af = full_herm(A)
        assert sl.potrf(A) == 0
        F = D(A)
        if uplo == Uplo.Lower:
            L = torch.tril(F)
            close(L @ L.mH, Af, 1e-12)
        else:
            U = torch.triu(F)
            close(U.mH @ U, Af, 1e-12)
    B = mat(n, 5, nb, 12, p, q, dt)
    Bd = D(B)
    sl.potrs(A, B)
    close(Af @ D(B), Bd, 1e-10)


def check_lu(p, q, dt=torch.float64):
    n, nb = 90, 16
    A = mat(n, n, nb, 13, p, q, dt)
    Ad = D(A)
    piv = sl.Pivots()
    B = mat(n, 4, nb, 14, p, q, dt)
    Bd = D(B)
    assert sl.gesv(A, piv, B) == 0
    X = D(B)
    close(Ad @ X, Bd, 1e-10)
    # factor property P A = L U
    F = D(A)
    L = torch.tril(F, -1) + torch.eye(n, dtype=dt)
    U = torch.triu(F)
    PA = Ad.clone()
    for i, pv in enumerate(piv.ipiv.tolist()):
        if pv != i:
            PA[[i, pv]] = PA[[pv, i]]
    close(L @ U, PA, 1e-12)


def _lu_check(Ad, F, piv, m, n, dt, tol=1e-12):
    k = min(m, n)
    L = torch.tril(F[:, :k], -1) + torch.eye(m, k, dtype=dt)
    U = torch.triu(F[:k, :])
    PA = Ad.clone()
    for i, pv in enumerate(piv.ipiv.tolist()):
        if pv != i:
            PA[[i, pv]] = PA[[pv, i]]
    close(L @ U, PA, tol)
    return L


def check_lu_methods(p, q, dt=torch.float64):
    """getrf partial pivoting / CALU / no pivoting on non-square shapes and
    lookahead depths; the distributed row exchange (swap plan + column
    all-reduce) and the tournament both run on every grid."""
    from slate_amd.core.enums import MethodLU, Option
    for (m, n, la) in [(100, 70, 0), (64, 96, 2), (83, 83, 1)]:
        A = mat(m, n, 16, 31, p, q, dt)
        Ad = D(A)
        piv = sl.Pivots()
        assert sl.getrf(A, piv, {Option.Lookahead: la}) == 0
        if p > 1:
            # exact point-to-point row exchange: per step,
            # the bytes this rank sends are at most (rows that change
            # process row) x (local columns) x element size
            from slate_amd.models import lu as _lu
            es = torch.empty(0, dtype=dt).element_size()
            for rec in _lu.XCHG_STATS:
                assert rec["bytes_sent"] <= rec["rows_cross"] * A.storage.bc.nloc * es, rec
            import torch.distributed as dist
            cnt = torch.tensor([len(_lu.XCHG_STATS)])
            dist.all_reduce(cnt)
            assert int(cnt) > 0
        L = _lu_check(Ad, D(A), piv, m, n, dt)
        assert L.abs().max().item() <= 1.0 + 1e-12          # partial pivoting: |L| <= 1
    # CALU with small leaves (several play-off rounds per rank)
    import os
    os.environ["SLATE_AMD_CALU_LEAF"] = "16"
    try:
        for (m, n) in [(120, 80), (80, 80), (96, 60), (60, 96)]:   # short last panels, both ways
            A = mat(m, n, 16, 32, p, q, dt)
            Ad = D(A)
            piv = sl.Pivots()
            assert sl.getrf(A, piv, {Option.MethodLU: MethodLU.CALU}) == 0
            L = _lu_check(Ad, D(A), piv, m, n, dt, 1e-11)
            assert L.abs().max().item() < 10.0                   # tournament: bounded growth
            B = mat(m, 3, 16, 33, p, q, dt)
            if m == n and m % 16 == 0:
                Bd = D(B)
                sl.getrs(A, piv, B)
                close(Ad @ D(B), Bd, 1e-10)
    finally:
        del os.environ["SLATE_AMD_CALU_LEAF"]
    # no pivoting on a diagonally dominant matrix
    A = mat(80, 80, 16, 34, p, q, dt)
    Ad = D(A) + 80 * torch.eye(80, dtype=dt)
    sl.from_dense(A, Ad)
    assert sl.getrf_nopiv(A) == 0
    F = D(A)
    close((torch.tril(F, -1) + torch.eye(80, dtype=dt)) @ torch.triu(F), Ad, 1e-12)
    # transposed solve exercises the backward permutation
    A = mat(64, 64, 16, 35, p, q, dt)
    Ad = D(A)
    piv = sl.Pivots()
    assert sl.getrf(A, piv) == 0
    B = mat(64, 2, 16, 36, p, q, dt)
    Bd = D(B)
    sl.getrs(A.transpose(), piv, B)
    close(Ad.T @ D(B), Bd, 1e-10)


def check_norms(p, q, dt=torch.float64):
    A = mat(77, 55, 16, 15, p, q, dt)
    Ad = D(A)
    for nt, ref in [(Norm.Max, Ad.abs().max()), (Norm.One, Ad.abs().sum(0).max()),
                    (Norm.Inf, Ad.abs().sum(1).max()), (Norm.Fro, torch.linalg.norm(Ad))]:
        v = sl.norm(nt, A)
        assert abs(float(v) - ref.item()) < 1e-10 * max(1.0, ref.item()), (nt, float(v), ref.item())
    H = herm(50, 16, 16, p, q, dt)
    Hf = full_herm(H)
    assert abs(float(sl.norm(Norm.One, H)) - Hf.abs().sum(0).max().item()) < 1e-9


def check_aux(p, q, dt=torch.float64):
    A = mat(40, 30, 16, 17, p, q, dt)
    B = mat(40, 30, 16, 18, p, q, dt)
    Ad, Bd = D(A), D(B)
    sl.add(2.0, A, -1.0, B)
    close(D(B), 2.0 * Ad - Bd)
    sl.scale(3.0, 2.0, A)
    close(D(A), 1.5 * Ad)
    sl.set(0.5, 2.0, A)
    E = torch.full((40, 30), 0.5, dtype=dt)
    E.diagonal().fill_(2.0)
    close(D(A), E)
    C = sl.Matrix(40, 30, nb=8, p=q, q=p, dtype=dt)
    C.insertLocalTiles()
    sl.redistribute(B, C)
    close(D(C), D(B))


ALL = [check_gemm, check_herk_trsm_trmm, check_potrf, check_lu, check_lu_methods, check_norms, check_aux]


def _run_all(rank, size, p, q):
    for f in ALL:
        f(p, q)
    check_potrf(p, q, uplo=Uplo.Upper)
    check_lu(p, q, torch.complex128)
    check_gemm(p, q, torch.complex128)


# ----------------------------------------------------------------- tests
@pytest.mark.parametrize("check", ALL, ids=lambda f: f.__name__)
def test_single_rank(check):
    check(1, 1)


def test_single_rank_complex():
    check_gemm(1, 1, torch.complex128)
    check_potrf(1, 1, torch.complex128)
    check_potrf(1, 1, torch.complex128, Uplo.Upper)
    check_lu(1, 1, torch.complex128)
    check_herk_trsm_trmm(1, 1, torch.complex128)


@pytest.mark.parametrize("grid", [(2, 1), (1, 2)])
def test_two_ranks(grid):
    run_dist(_run_all, 2, *grid)


def test_four_ranks():
    run_dist(_run_all, 4, 2, 2)


def check_qr(p, q, dt=torch.float64):
    from slate_amd.core.enums import Option
    m, n, nb = 300, 120, 16
    A = mat(m, n, nb, 21, p, q, dt)
    A0 = D(A)
    T = sl.TriangularFactors()
    sl.geqrf(A, T, {Option.Lookahead: 2})
    R = torch.triu(D(A))[:n]
    close(R.mH @ R, A0.mH @ A0, 1e-12)
    B = mat(m, 3, nb, 22, p, q, dt)
    Bd = D(B)
    sl.gels(mat(m, n, nb, 21, p, q, dt), sl.TriangularFactors(), B)
    close(D(B)[:n], torch.linalg.lstsq(A0, Bd).solution, 1e-9)


def _run_8(rank, size, p, q):
    for f in (check_gemm, check_potrf, check_lu, check_lu_methods, check_qr):
        f(p, q)


def _potrf_bcast_granularity(rank, size, p, q):
    """on the 2 x 4 grid, the first lookahead GEMM of a
    step waits for at most one tile row of the panel's row broadcast plus
    the lookahead tiles' column broadcast -- the equivalent of <= 4 MB at
    nb = 512 -- not for the whole nrow x kb panel; the rest of the row
    broadcast travels in several tile-granular messages behind it."""
    from slate_amd.models import chol
    n, nb = 2048, 128
    A = herm(n, nb, 31, p, q, torch.float64, Uplo.Lower)
    Af = full_herm(A)
    assert sl.potrf(A, {sl.Option.Lookahead: 1}) == 0
    L = torch.tril(D(A))
    close(L @ L.mH, Af, 1e-12)
    lim = 2 * nb * nb * 8                     # = 4 MB at nb = 512
    st = chol.POTRF_BCAST_STATS
    assert st and all(s["row_bytes_first"] + s["col_bytes_first"] <= lim for s in st), st
    early = st[0]
    assert early["row_bytes"] > lim, early     # the panel itself is larger ...
    assert early["row_msgs"] >= 3, early       # ... and goes in several messages


def _lu_no_panel_allgather(rank, size, p, q):
    """with p > 1 the partial-pivoting panel rows stay
    on their owners -- the only all-gathers are the per-column records
    (p (2b + 3) scalars); no rank receives another rank's m x nb panel."""
    from slate_amd.models import lu as lu_mod
    from slate_amd.parallel.comm import Comm
    seen = []
    orig = Comm.allgather

    def spy(self, t):
        seen.append(t.numel() * t.element_size())
        return orig(self, t)

    n, nb = 640, 64
    A = mat(n, n, nb, 41, p, q, torch.float64)
    A0 = D(A)
    Comm.allgather = spy
    try:
        piv = sl.Pivots()
        assert sl.getrf(A, piv, {sl.Option.Lookahead: 1}) == 0
    finally:
        Comm.allgather = orig
    F = D(A)
    L = torch.tril(F, -1) + torch.eye(n, dtype=F.dtype)
    U = torch.triu(F)
    perm = list(range(n))
    for i, j in enumerate(piv.ipiv.tolist()):
        perm[i], perm[j] = perm[j], perm[i]
    close(L @ U, A0[torch.as_tensor(perm)], 1e-12)
    b = 32
    assert seen and max(seen) <= (2 * b + 3) * 8, max(seen)       # one record per call, never a panel
    assert lu_mod.LU_DIST_STATS["columns"] > 0


def test_lu_distributed_panel_2x4():
    run_dist(_lu_no_panel_allgather, 8, 2, 4, timeout=600)


def test_potrf_tile_granular_bcast_2x4(monkeypatch):
    monkeypatch.setenv("SLATE_AMD_POTRF_CHUNK", "4")    # the mechanism (default 16: fewer, larger messages)
    run_dist(_potrf_bcast_granularity, 8, 2, 4, timeout=600)


@pytest.mark.parametrize("grid", [(2, 4), (1, 8), (8, 1)], ids=lambda g: f"{g[0]}x{g[1]}")
def test_eight_ranks(grid):
    """The 8-GPU node's grids (BASELINE: 2x4), rehearsed with 8 gloo ranks."""
    run_dist(_run_8, 8, *grid, timeout=600)


def _potrf_pairs(rank, size, p, q):
    check_potrf(p, q)
    check_potrf(p, q, torch.complex128)


@pytest.mark.parametrize("grid", [(1, 2), (2, 1), (2, 2)], ids=lambda g: f"{g[0]}x{g[1]}")
def test_potrf_step_pairs(grid, monkeypatch):
    """SLATE_AMD_POTRF_PAIR=1 (chol.py): the deferred K = 2 nb trailing
    update, odd and even tile counts, real and complex."""
    monkeypatch.setenv("SLATE_AMD_POTRF_PAIR", "1")
    run_dist(_potrf_pairs, grid[0] * grid[1], *grid)
