"""Band (gbsv, pbsv, gbmm, hbmm, tbsm) and indefinite (hesv) drivers
(reference: test_gbsv.cc, test_pbsv.cc, test_gbmm.cc, test_hbmm.cc,
test_tbsm.cc, test_hesv.cc)."""
import pytest
import torch

import slate_amd as sl
from slate_amd.models.aux import allgather_dense as D
from slate_amd.models.eig import _dense_hermitian

from dist_util import run_dist


def check_band(p=1, q=1, dt=torch.float64):
    n, nb, kl, ku = 150, 32, 20, 15
    A = sl.BandMatrix(n, n, kl, ku, nb=nb, p=p, q=q, dtype=dt)
    A.insertLocalTiles()
    sl.generate_matrix(A, "rands", 1)
    sl.band_mask(A)
    A0 = D(A).clone()
    i = torch.arange(n)
    dd = i[:, None] - i[None, :]
    assert A0[(dd > kl) | (dd < -ku)].abs().max() == 0
    B = sl.Matrix(n, 3, nb=nb, p=p, q=q, dtype=dt)
    B.insertLocalTiles()
    sl.generate_matrix(B, "rands", 2)
    B0 = D(B).clone()
    # gbmm
    C = sl.Matrix(n, 3, nb=nb, p=p, q=q, dtype=dt)
    C.insertLocalTiles()
    sl.generate_matrix(C, "rands", 3)
    C0 = D(C).clone()
    sl.gbmm(2.0, A, B, 0.5, C)
    assert (D(C) - (2 * A0 @ B0 + 0.5 * C0)).abs().max() < 1e-12
    # gbsv
    piv = sl.Pivots()
    assert sl.gbsv(A, piv, B) == 0
    assert (A0 @ D(B) - B0).abs().max() < 1e-11
    # pbsv
    H = sl.HermitianBandMatrix(sl.Uplo.Lower, n, 17, nb=nb, p=p, q=q, dtype=dt)
    H.insertLocalTiles()
    sl.generate_matrix(H, "poev", 4)
    sl.band_mask(H, 17, 0)
    Hf = _dense_hermitian(H)
    B2 = sl.Matrix(n, 2, nb=nb, p=p, q=q, dtype=dt)
    B2.insertLocalTiles()
    sl.generate_matrix(B2, "rands", 5)
    B2d = D(B2).clone()
    assert sl.pbsv(H, B2) == 0
    assert (Hf @ D(B2) - B2d).abs().max() < 1e-12


def check_indef(p=1, q=1, dt=torch.float64):
    n, nb = 120, 32
    S = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb, p=p, q=q, dtype=dt)
    S.insertLocalTiles()
    sl.generate_matrix(S, "rands", 5)
    Sf = _dense_hermitian(S)
    B = sl.Matrix(n, 3, nb=nb, p=p, q=q, dtype=dt)
    B.insertLocalTiles()
    sl.generate_matrix(B, "rands", 6)
    Bd = D(B).clone()
    assert sl.hesv(S, sl.Pivots(), None, None, None, B) == 0
    assert (Sf @ D(B) - Bd).abs().max() / (Sf.abs().max() * n) < 1e-13


@pytest.mark.parametrize("dt", [torch.float64, torch.complex128])
def test_band(dt):
    check_band(dt=dt)


@pytest.mark.parametrize("dt", [torch.float64, torch.complex128])
def test_hesv(dt):
    check_indef(dt=dt)


def test_tbsm_hbmm():
    n, nb, kd = 100, 16, 9
    T = sl.TriangularBandMatrix(sl.Uplo.Lower, sl.Diag.NonUnit, n, kd, nb=nb)
    T.insertLocalTiles()
    sl.generate_matrix(T, "rands", 7)
    sl.band_mask(T, kd, 0)
    Td = torch.tril(D(T)) + 4 * torch.eye(n, dtype=torch.float64)
    sl.from_dense(T, Td)
    B = sl.Matrix(n, 4, nb=nb)
    B.insertLocalTiles()
    sl.generate_matrix(B, "rands", 8)
    Bd = D(B).clone()
    sl.tbsm(sl.Side.Left, 1.0, T, B)
    assert (Td @ D(B) - Bd).abs().max() < 1e-12
    H = sl.HermitianBandMatrix(sl.Uplo.Lower, n, kd, nb=nb)
    H.insertLocalTiles()
    sl.generate_matrix(H, "rands", 9)
    sl.band_mask(H, kd, 0)
    Hf = _dense_hermitian(H)
    C = sl.Matrix(n, 4, nb=nb)
    C.insertLocalTiles()
    sl.hbmm(sl.Side.Left, 1.0, H, B, 0.0, C)
    assert (D(C) - Hf @ D(B)).abs().max() < 1e-12


def _dist(rank, size, p, q):
    check_band(p, q)
    check_indef(p, q)
    check_hetrf_dist(p, q)
    check_band_products(p, q)


def check_band_products(p=1, q=1):
    """gbmm (all ops) and hbmm (both sides, both triangles) on any grid:
    point-to-point band products (no replicated B, no all-reduced C)."""
    for dt in (torch.float64, torch.complex128):
        n, nb, kl, ku = 90, 16, 20, 11
        A = sl.BandMatrix(n, n, kl, ku, nb=nb, p=p, q=q, dtype=dt)
        A.insertLocalTiles()
        sl.generate_matrix(A, "rands", 31)
        sl.band_mask(A)
        Ad = D(A)
        for op in (sl.Op.NoTrans, sl.Op.Trans, sl.Op.ConjTrans):
            B = sl.Matrix(n, 7, nb=nb, p=p, q=q, dtype=dt)
            B.insertLocalTiles()
            sl.generate_matrix(B, "rands", 32)
            C = sl.Matrix(n, 7, nb=nb, p=p, q=q, dtype=dt)
            C.insertLocalTiles()
            sl.generate_matrix(C, "rands", 33)
            Bd, Cd = D(B), D(C)
            Av = A if op == sl.Op.NoTrans else (A.transpose() if op == sl.Op.Trans else A.conj_transpose())
            Ao = Ad if op == sl.Op.NoTrans else (Ad.T if op == sl.Op.Trans else Ad.mH)
            sl.gbmm(2.0, Av, B, 0.5, C)
            assert (D(C) - (2.0 * Ao @ Bd + 0.5 * Cd)).abs().max() < 1e-12
        for uplo in (sl.Uplo.Lower, sl.Uplo.Upper):
            H = sl.HermitianBandMatrix(uplo, n, 13, nb=nb, p=p, q=q, dtype=dt)
            H.insertLocalTiles()
            sl.generate_matrix(H, "rands", 34)
            sl.band_mask(H, 13, 0) if uplo == sl.Uplo.Lower else sl.band_mask(H, 0, 13)
            Hf = _dense_hermitian(H)
            for side in (sl.Side.Left, sl.Side.Right):
                B = sl.Matrix(n, 5, nb=nb, p=p, q=q, dtype=dt) if side == sl.Side.Left else \
                    sl.Matrix(5, n, nb=nb, p=p, q=q, dtype=dt)
                B.insertLocalTiles()
                sl.generate_matrix(B, "rands", 35)
                C = sl.Matrix(B.m(), B.n(), nb=nb, p=p, q=q, dtype=dt)
                C.insertLocalTiles()
                sl.generate_matrix(C, "rands", 36)
                Bd, Cd = D(B), D(C)
                sl.hbmm(side, 1.5, H, B, -1.0, C)
                ref = 1.5 * (Hf @ Bd if side == sl.Side.Left else Bd @ Hf) - Cd
                assert (D(C) - ref).abs().max() < 1e-12


def test_band_products_one_rank():
    check_band_products()


def _dist_prod(rank, size):
    check_band_products(1, size)


def test_band_products_four_ranks():
    run_dist(_dist_prod, 4)


def check_hetrf_dist(p, q):
    """Distributed Aasen (models/hetrf_dist.py): zero diagonal (pivoting
    needed), padded orders, both uplos, complex; P A P^H = L T L^H from the
    grid factors and hesv residuals -- no rank gathers A."""
    from slate_amd.models.hetrf import _blk
    for dt, uplo, n, nb in [(torch.float64, sl.Uplo.Lower, 70, 16), (torch.complex128, sl.Uplo.Upper, 45, 8),
                            (torch.float64, sl.Uplo.Upper, 64, 16)]:
        S = sl.HermitianMatrix(uplo, n, nb=nb, p=p, q=q, dtype=dt)
        S.insertLocalTiles()
        sl.generate_matrix(S, "rands", 21)
        Sf = _dense_hermitian(S)
        Sf = Sf - torch.diag(torch.diagonal(Sf))
        sl.from_dense(S, torch.tril(Sf) if uplo == sl.Uplo.Lower else torch.triu(Sf))
        B = sl.Matrix(n, 3, nb=nb, p=p, q=q, dtype=dt)
        B.insertLocalTiles()
        sl.generate_matrix(B, "rands", 22)
        Bd = D(B).clone()
        piv = sl.Pivots()
        assert sl.hetrf(S, piv) == 0
        F = S._hetrf
        if p * q > 1:
            assert getattr(F, "distributed", False)
        N, k = F.N, F.N // F.nb
        T = torch.zeros(N, N, dtype=dt)
        for J in range(k):
            T[J * F.nb:(J + 1) * F.nb, J * F.nb:(J + 1) * F.nb] = _blk(F.Td, J, F.nb).cpu()
            if J + 1 < k:
                T[(J + 1) * F.nb:(J + 2) * F.nb, J * F.nb:(J + 1) * F.nb] = _blk(F.Tl, J + 1, F.nb).cpu()
                T[J * F.nb:(J + 1) * F.nb, (J + 1) * F.nb:(J + 2) * F.nb] = _blk(F.Tl, J + 1, F.nb).cpu().mH
        Ap = torch.eye(N, dtype=dt)
        Ap[:n, :n] = Sf
        pm = torch.as_tensor(F.perm).cpu()
        L = (D(F.L) if hasattr(F.L, "storage") else F.L).cpu()
        assert ((L @ T @ L.mH - Ap[pm][:, pm]).abs().max() / Sf.abs().max()).item() < 1e-12
        sl.hetrs(S, piv, None, None, B)
        assert (Sf @ D(B) - Bd).abs().max() / (Sf.abs().max() * D(B).abs().max() * n) < 1e-13


def _dist_hetrf(rank, size, p, q):
    check_hetrf_dist(p, q)


@pytest.mark.parametrize("grid", [(2, 2), (2, 4)])
def test_hetrf_distributed_grids(grid):
    run_dist(_dist_hetrf, grid[0] * grid[1], *grid)


@pytest.mark.parametrize("grid", [(2, 1), (1, 2)])
def test_band_indef_distributed(grid):
    run_dist(_dist, 2, *grid)


@pytest.mark.gpu
def test_band_gpu():
    dev = torch.device("cuda")
    n, nb, kl, ku = 1000, 128, 60, 40
    A = sl.BandMatrix(n, n, kl, ku, nb=nb, device=dev)
    A.insertLocalTiles(device=0)
    sl.generate_matrix(A, "rands", 1)
    sl.band_mask(A)
    A0 = D(A).clone()
    B = sl.Matrix(n, 3, nb=nb, device=dev)
    B.insertLocalTiles(device=0)
    sl.generate_matrix(B, "rands", 2)
    B0 = D(B).clone()
    assert sl.gbsv(A, sl.Pivots(), B) == 0
    assert (A0 @ D(B) - B0).abs().max().item() < 1e-10


def _tri_band(uplo, diag, n, kd, nb, dt, seed, p=1, q=1):
    T = sl.TriangularBandMatrix(uplo, diag, n, kd, nb=nb, p=p, q=q, dtype=dt)
    T.insertLocalTiles()
    sl.generate_matrix(T, "rands", seed)
    lo = uplo == sl.Uplo.Lower
    sl.band_mask(T, kd if lo else 0, 0 if lo else kd)
    Td = D(T)
    Td = Td + 4 * torch.eye(n, dtype=dt)
    sl.from_dense(T, Td)
    Td = torch.tril(Td) if lo else torch.triu(Td)
    if diag == sl.Diag.Unit:
        Td = Td - torch.diag(torch.diagonal(Td)) + torch.eye(n, dtype=dt)
    return T, Td


def check_band_full(p=1, q=1, dt=torch.float64):
    """Compact storage + every band driver variant on a grid."""
    n, nb = 133, 16
    kl, ku = 21, 9
    A = sl.BandMatrix(n, n, kl, ku, nb=nb, p=p, q=q, dtype=dt)
    A.insertLocalTiles()
    sl.generate_matrix(A, "rands", 11)
    sl.band_mask(A)
    # storage is O(n (kl + ku)): slab rows = (ceil(kl/nb) + ceil((kl+ku)/nb) + 1) nb
    s = A.storage
    assert s.get_slab(s.band_slot()).shape[0] == (2 + 2 + 1) * nb
    A0 = D(A).clone()
    # gbmm with op(A) = A^T and A^H
    B = sl.Matrix(n, 5, nb=nb, p=p, q=q, dtype=dt)
    B.insertLocalTiles()
    sl.generate_matrix(B, "rands", 12)
    B0 = D(B).clone()
    for view, ref in ((A.transpose(), A0.mT), (A.conj_transpose(), A0.mH)):
        C = sl.Matrix(n, 5, nb=nb, p=p, q=q, dtype=dt)
        C.insertLocalTiles()
        sl.generate_matrix(C, "rands", 13)
        C0 = D(C).clone()
        sl.gbmm(1.5, view, B, -1.0, C)
        assert (D(C) - (1.5 * ref @ B0 - C0)).abs().max() < 1e-11
    # gbtrf / gbtrs, then tbsm with the pivots on the unit-lower factor
    piv = sl.Pivots()
    assert sl.gbtrf(A, piv) == 0
    X = sl.Matrix(n, 5, nb=nb, p=p, q=q, dtype=dt)
    X.insertLocalTiles()
    sl.copy(B, X)
    sl.gbtrs(A, piv, X)
    assert (A0 @ D(X) - B0).abs().max() < 1e-10
    Lf = sl.TriangularBandMatrix(sl.Uplo.Lower, sl.Diag.Unit, matrix=A, kd=kl)
    Uf = sl.TriangularBandMatrix(sl.Uplo.Upper, sl.Diag.NonUnit, matrix=A, kd=kl + ku)
    Y = sl.Matrix(n, 5, nb=nb, p=p, q=q, dtype=dt)
    Y.insertLocalTiles()
    sl.copy(B, Y)
    sl.tbsm(sl.Side.Left, 1.0, Lf, Y, piv)
    sl.tbsm(sl.Side.Left, 1.0, Uf, Y)
    assert (D(Y) - D(X)).abs().max() < 1e-10
    # tbsm: all uplo x op x diag, left and right
    for uplo in (sl.Uplo.Lower, sl.Uplo.Upper):
        for diag in (sl.Diag.NonUnit, sl.Diag.Unit):
            T, Td = _tri_band(uplo, diag, n, 13, nb, dt, 14, p, q)
            for view, ref in ((T, Td), (T.transpose(), Td.mT), (T.conj_transpose(), Td.mH)):
                Z = sl.Matrix(n, 3, nb=nb, p=p, q=q, dtype=dt)
                Z.insertLocalTiles()
                sl.generate_matrix(Z, "rands", 15)
                Z0 = D(Z).clone()
                sl.tbsm(sl.Side.Left, 2.0, view, Z)
                Zd = D(Z)
                assert (ref @ Zd - 2.0 * Z0).abs().max() / (ref.abs().max() * Zd.abs().max() * n) < 1e-15, \
                    (uplo, diag)
                W = sl.Matrix(4, n, nb=nb, p=p, q=q, dtype=dt)
                W.insertLocalTiles()
                sl.generate_matrix(W, "rands", 16)
                W0 = D(W).clone()
                sl.tbsm(sl.Side.Right, 1.0, view, W)
                Wd = D(W)
                assert (Wd @ ref - W0).abs().max() / (ref.abs().max() * Wd.abs().max() * n) < 1e-15, \
                    (uplo, diag, "R")
    # pbsv Upper, hbmm Right
    kd = 11
    H = sl.HermitianBandMatrix(sl.Uplo.Upper, n, kd, nb=nb, p=p, q=q, dtype=dt)
    H.insertLocalTiles()
    sl.generate_matrix(H, "poev", 17)
    sl.band_mask(H, 0, kd)
    Hf = _dense_hermitian(H)
    Wr = sl.Matrix(6, n, nb=nb, p=p, q=q, dtype=dt)
    Wr.insertLocalTiles()
    sl.generate_matrix(Wr, "rands", 18)
    Cr = sl.Matrix(6, n, nb=nb, p=p, q=q, dtype=dt)
    Cr.insertLocalTiles()
    sl.hbmm(sl.Side.Right, 1.0, H, Wr, 0.0, Cr)
    assert (D(Cr) - D(Wr) @ Hf).abs().max() < 1e-11
    Bh = sl.Matrix(n, 2, nb=nb, p=p, q=q, dtype=dt)
    Bh.insertLocalTiles()
    sl.generate_matrix(Bh, "rands", 19)
    Bh0 = D(Bh).clone()
    assert sl.pbsv(H, Bh) == 0
    assert (Hf @ D(Bh) - Bh0).abs().max() < 1e-11
    U = torch.triu(D(H))
    assert (U.mH @ U - Hf).abs().max() < 1e-10 * Hf.abs().max()


@pytest.mark.parametrize("dt", [torch.float64, torch.complex128])
def test_band_full(dt):
    check_band_full(dt=dt)


def _band_full_dist(rank, size, p, q):
    check_band_full(p, q)
    check_band_full(p, q, torch.complex128)


@pytest.mark.parametrize("nranks", [2, 3, 4])
def test_band_full_distributed(nranks):
    """Band storage is 1-D column-cyclic over all ranks whatever p x q."""
    run_dist(_band_full_dist, nranks, 1, nranks)


def _band_norms(rank, size, p, q):
    n, nb = 90, 16
    A = sl.BandMatrix(n, n, 13, 7, nb=nb, p=p, q=q)
    A.insertLocalTiles()
    sl.generate_matrix(A, "rands", 3)
    sl.band_mask(A)
    Ad = D(A)
    H = sl.HermitianBandMatrix(sl.Uplo.Lower, n, 10, nb=nb, p=p, q=q)
    H.insertLocalTiles()
    sl.generate_matrix(H, "rands", 4)
    sl.band_mask(H, 10, 0)
    Hd = _dense_hermitian(H)
    for nt, f in ((sl.Norm.Max, lambda X: X.abs().max()), (sl.Norm.One, lambda X: X.abs().sum(0).max()),
                  (sl.Norm.Inf, lambda X: X.abs().sum(1).max()), (sl.Norm.Fro, lambda X: X.norm())):
        assert abs(sl.norm(nt, A) - float(f(Ad))) < 1e-12 * float(f(Ad))
        assert abs(sl.norm(nt, H) - float(f(Hd))) < 1e-12 * float(f(Hd)), nt


@pytest.mark.parametrize("nranks", [1, 3])
def test_band_norms(nranks):
    """Norms straight from the compact band tiles (no dense gather)."""
    if nranks == 1:
        _band_norms(0, 1, 1, 1)
    else:
        run_dist(_band_norms, nranks, 1, nranks)


@pytest.mark.gpu
def test_band_full_gpu():
    """Compact band storage on the GPU: pbsv, tbsm, gbmm, hbmm (slab GEMMs)."""
    dev = torch.device("cuda")
    n, nb, kd = 1500, 128, 100
    H = sl.HermitianBandMatrix(sl.Uplo.Lower, n, kd, nb=nb, device=dev)
    H.insertLocalTiles(device=0)
    sl.generate_matrix(H, "poev", 4)
    sl.band_mask(H, kd, 0)
    Hf = _dense_hermitian(H)
    B = sl.Matrix(n, 4, nb=nb, device=dev)
    B.insertLocalTiles(device=0)
    sl.generate_matrix(B, "rands", 5)
    B0 = D(B).clone()
    C = sl.Matrix(n, 4, nb=nb, device=dev)
    C.insertLocalTiles(device=0)
    sl.hbmm(sl.Side.Left, 1.0, H, B, 0.0, C)
    assert ((D(C) - Hf @ B0).abs().max() / (Hf.abs().max() * n)).item() < 1e-14
    assert sl.pbsv(H, B) == 0
    assert ((Hf @ D(B) - B0).abs().max() / (Hf.abs().max() * n)).item() < 1e-14


@pytest.mark.parametrize("dt,uplo,n,nb", [(torch.float64, sl.Uplo.Lower, 200, 16),
                                           (torch.complex128, sl.Uplo.Upper, 77, 8),
                                           (torch.float64, sl.Uplo.Upper, 64, 16)])
def test_hetrf_blocked_aasen(dt, uplo, n, nb):
    """Blocked Aasen: P A P^H = L T L^H with T block tridiagonal, on a
    matrix with a zero diagonal (pivoting required), padded orders."""
    from slate_amd.models.hetrf import _blk
    S = sl.HermitianMatrix(uplo, n, nb=nb, dtype=dt)
    S.insertLocalTiles()
    sl.generate_matrix(S, "rands", 21)
    Sf = _dense_hermitian(S)
    Sf = Sf - torch.diag(torch.diagonal(Sf))          # zero diagonal: indefinite, needs pivots
    sl.from_dense(S, torch.tril(Sf) if uplo == sl.Uplo.Lower else torch.triu(Sf))
    B = sl.Matrix(n, 4, nb=nb, dtype=dt)
    B.insertLocalTiles()
    sl.generate_matrix(B, "rands", 22)
    Bd = D(B).clone()
    piv = sl.Pivots()
    assert sl.hetrf(S, piv) == 0
    F = S._hetrf
    N, k = F.N, F.N // F.nb
    T = torch.zeros(N, N, dtype=dt)
    for J in range(k):
        T[J * F.nb:(J + 1) * F.nb, J * F.nb:(J + 1) * F.nb] = _blk(F.Td, J, F.nb).cpu()
        if J + 1 < k:
            T[(J + 1) * F.nb:(J + 2) * F.nb, J * F.nb:(J + 1) * F.nb] = _blk(F.Tl, J + 1, F.nb).cpu()
            T[J * F.nb:(J + 1) * F.nb, (J + 1) * F.nb:(J + 2) * F.nb] = _blk(F.Tl, J + 1, F.nb).cpu().mH
    Ap = torch.eye(N, dtype=dt)
    Ap[:n, :n] = Sf
    p = F.perm.cpu()
    L = F.L.cpu()
    assert ((L @ T @ L.mH - Ap[p][:, p]).abs().max() / Sf.abs().max()).item() < 1e-12
    # partial pivoting: |l| <= 1 (real); cabs1 pivot choice bounds |l| by sqrt(2) (complex)
    assert L.abs().max().item() <= (2 ** 0.5 if L.is_complex() else 1.0) + 1e-12
    sl.hetrs(S, piv, None, None, B)
    assert (Sf @ D(B) - Bd).abs().max() / (Sf.abs().max() * D(B).abs().max() * n) < 1e-13


@pytest.mark.gpu
def test_hesv_gpu():
    """Blocked Aasen on the GPU (batched MFMA GEMMs, GPU LU panel, band T)."""
    dev = torch.device("cuda")
    n, nb = 1000, 64
    S = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb, device=dev)
    S.insertLocalTiles(device=0)
    sl.generate_matrix(S, "rands", 5)
    Sf = _dense_hermitian(S)
    B = sl.Matrix(n, 3, nb=nb, device=dev)
    B.insertLocalTiles(device=0)
    sl.generate_matrix(B, "rands", 6)
    Bd = D(B).clone()
    assert sl.hesv(S, sl.Pivots(), None, None, None, B) == 0
    X = D(B)
    assert ((Sf @ X - Bd).abs().max() / (Sf.abs().max() * X.abs().max() * n)).item() < 1e-13


def _band_solve_workspace(rank, size, p, q):
    from slate_amd.models import band as BM
    n, nb, kl, ku, nrhs = 257, 16, 21, 9, 7
    A = sl.BandMatrix(n, n, kl, ku, nb=nb, p=p, q=q)
    A.insertLocalTiles()
    sl.generate_matrix(A, "rands", 31)
    sl.band_mask(A)
    A0 = D(A).clone()
    B = sl.Matrix(n, nrhs, nb=nb, p=p, q=q)
    B.insertLocalTiles()
    sl.generate_matrix(B, "rands", 32)
    B0 = D(B).clone()
    piv = sl.Pivots()
    assert sl.gbsv(A, piv, B) == 0
    X = D(B)
    assert (A0 @ X - B0).abs().max() / (A0.abs().max() * X.abs().max() * n) < 1e-15
    st = BM.BAND_SOLVE_STATS
    # one window of (kb + bandwidth) rows and this rank's tile rows -- never
    # the n x nrhs right-hand side
    assert st["window_elems"] <= (nb + kl + (kl + ku) + nb) * nrhs, st
    assert st["local_elems"] <= -(-(-(-n // nb)) // size) * nb * nrhs, st
    assert st["window_elems"] + st["local_elems"] < n * nrhs, st


def test_band_solve_no_rhs_replication_8_ranks():
    """gbtrs / pbtrs / tbsm keep the right-hand side 1-D row-cyclic; each
    step gathers only its window onto the factor column's owner."""
    run_dist(_band_solve_workspace, 8, 2, 4)
