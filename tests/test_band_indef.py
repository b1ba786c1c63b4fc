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
