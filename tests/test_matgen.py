"""Matrix generator (SLATE matgen/generate_matrix_ge.cc, generate_matrix_utils.cc):
gallery kinds against independent closed forms, spectral kinds (svd / poev
/ heev / diag with distributions and cond) on grids, scalings, modifiers,
grid independence."""
import math

import numpy as np
import pytest
import torch

import slate_amd as sl
from slate_amd.models.aux import allgather_dense as D
from slate_amd.models.eig import _dense_hermitian

from dist_util import run_dist


def _ref(kind, m, n):
    """Independent numpy definitions (Matlab gallery / SLATE docs)."""
    i = np.arange(m)[:, None].astype(float)
    j = np.arange(n)[None, :].astype(float)
    N = max(m, n)
    d = i - j
    I, J = i + 1, j + 1
    if kind == "fiedler":
        return np.abs(d)
    if kind == "kms":
        return 0.5 ** np.abs(d)
    if kind == "circul":
        return (j - i) % N + 1
    if kind == "orthog":
        return math.sqrt(2 / (N + 1)) * np.sin(I * J * math.pi / (N + 1))
    if kind == "cauchy":
        return 1.0 / (I + J)
    if kind == "lotkin":
        return np.where(i == 0, 1.0, 1.0 / (I + J - 1))
    if kind == "pei":
        return np.where(d == 0, 2.0, 1.0)
    if kind == "tridiag":
        return np.where(d == 0, 2.0, np.where(np.abs(d) == 1, -1.0, 0.0))
    if kind == "triw":
        return np.where(d == 0, 1.0, np.where(d > 0, 0.0, -1.0))
    if kind == "chow":
        return np.where(d < -1, 0.0, 1.0)
    if kind == "gcdmat":
        return np.gcd(I.astype(int), J.astype(int)).astype(float)
    if kind == "redheff":
        return np.where((J % I == 0) | (j == 0), 1.0, 0.0)
    if kind == "riemann":
        return np.where((J + 1) % (I + 1) == 0, J, -1.0)
    if kind == "parter":
        return 1.0 / (d + 0.5)
    if kind == "clement":
        return np.where(d == 1, N - j - 1, np.where(d == -1, j, 0.0))
    if kind == "toeppen":
        return np.where(d == -1, 10.0, np.where(d == 1, -10.0, np.where(np.abs(d) == 2, 1.0, 0.0)))
    if kind == "jordanT":
        return np.where((d == 0) | (d == 1), 1.0, 0.0)
    if kind == "gfpp":
        return np.where(j == n - 1, 1.0, np.where(d > 0, -1.0, np.where(d == 0, 0.5, 0.0)))
    if kind == "ris":
        return 0.5 / (N - I - J + 1.5)
    if kind == "zielkeNS":
        return np.where(j < i, 1.0, np.where((i == 0) & (j == N - 1), -1.0, 0.0))
    raise KeyError(kind)


GALLERY = ["fiedler", "kms", "circul", "orthog", "cauchy", "lotkin", "pei", "tridiag", "triw", "chow", "gcdmat",
           "redheff", "riemann", "parter", "clement", "toeppen", "jordanT", "gfpp", "ris", "zielkeNS"]


@pytest.mark.parametrize("kind", GALLERY)
def test_gallery(kind):
    m, n = 23, 17
    A = sl.Matrix(m, n, nb=5)
    A.insertLocalTiles()
    sl.generate_matrix(A, kind)
    assert np.abs(D(A).numpy() - _ref(kind, m, n)).max() < 1e-13


def test_chebspec_stable():
    """chebspec (SLATE/Matlab chebspec(n, 1): Chebyshev differentiation on
    cos(pi (k+1) / n), boundary condition built in) has every eigenvalue in
    the open left half-plane."""
    n = 10
    A = sl.Matrix(n, n, nb=4)
    A.insertLocalTiles()
    sl.generate_matrix(A, "chebspec")
    ev = torch.linalg.eigvals(D(A))
    assert (ev.real < 0).all()


def _spectral(rank, size, p, q):
    m, n, nb = 50, 36, 8
    for dist in ("arith", "geo", "cluster0", "cluster1", "rgeo", "logrand"):
        A = sl.Matrix(m, n, nb=nb, p=p, q=q)
        A.insertLocalTiles()
        s = sl.generate_matrix(A, "svd_" + dist, 9, cond=1e4)
        sv = torch.linalg.svdvals(D(A))
        assert (sv - s.abs().sort(descending=True).values).abs().max() < 1e-12, dist
        if dist != "logrand":
            assert abs(sv[0] / sv[-1] / 1e4 - 1) < 1e-8, dist
    H = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb, p=p, q=q, dtype=torch.complex128)
    H.insertLocalTiles()
    w = sl.generate_matrix(H, "heev_arith", 3, cond=50.0)
    ev = torch.linalg.eigvalsh(_dense_hermitian(H))
    assert (ev - w.sort().values).abs().max() < 1e-12
    assert (w < 0).any() and (w > 0).any()
    P = sl.HermitianMatrix(sl.Uplo.Upper, n, nb=nb, p=p, q=q)
    P.insertLocalTiles()
    sl.generate_matrix(P, "poev_geo", 4, cond=1e3)
    ev = torch.linalg.eigvalsh(_dense_hermitian(P))
    assert ev.min() > 0 and abs(ev.max() / ev.min() / 1e3 - 1) < 1e-8
    G = sl.Matrix(n, n, nb=nb, p=p, q=q)
    G.insertLocalTiles()
    sl.generate_matrix(G, "diag_specified", 1, sigma=list(range(1, n + 1)))
    assert (D(G) - torch.diag(torch.arange(1, n + 1, dtype=torch.float64))).abs().max() == 0


def test_spectral_one_rank():
    _spectral(0, 1, 1, 1)


@pytest.mark.parametrize("grid", [(2, 2), (1, 3)], ids=lambda g: f"{g[0]}x{g[1]}")
def test_spectral_grid(grid):
    """Random unitary factors by the distributed QR: no rank holds A."""
    run_dist(_spectral, grid[0] * grid[1], *grid)


def test_scaling_modifiers_and_grid_independence():
    n = 30
    ref = None
    for nb in (4, 7, 30):
        A = sl.Matrix(n, n, nb=nb)
        A.insertLocalTiles()
        sl.generate_matrix(A, "randn_dominant_zerocol0.5", 11)
        Ad = D(A)
        ref = Ad if ref is None else ref
        assert (Ad - ref).abs().max() == 0                      # independent of the tiling
    c = round(0.5 * (n - 1))
    assert ref[:, c].abs().max() == 0
    off = ref.abs().sum(1) - ref.diagonal().abs()
    rows = torch.arange(n) != c
    assert (ref.diagonal().abs()[rows] > off[rows]).all()       # dominant
    A = sl.Matrix(n, n, nb=8)
    A.insertLocalTiles()
    sl.generate_matrix(A, "rands_large", 2)
    assert 1e150 < D(A).abs().max() < 1e155


def test_copy_general_into_hermitian():
    """Regression: copy(general, Hermitian) with identical layouts copies the
    stored triangle piece by piece (off-diagonal tiles included)."""
    n = 30
    M = sl.Matrix(n, n, nb=8)
    M.insertLocalTiles()
    sl.generate_matrix(M, "rands", 1)
    H = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=8)
    H.insertLocalTiles()
    sl.copy(M, H)
    assert (torch.tril(D(H)) - torch.tril(D(M))).abs().max() == 0
