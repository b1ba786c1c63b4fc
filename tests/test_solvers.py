"""Mixed precision (gesv_mixed[_gmres], posv_mixed[_gmres]), RBT, inverses
(getri, potri, trtri), condition estimates (reference: test_gesv.cc with
--method-gesv, test_posv.cc, test_getri.cc, test_potri.cc, test_gecondest.cc,
test_pocondest.cc, test_trcondest.cc)."""
import pytest
import torch

import slate_amd as sl
from slate_amd.core.enums import Option
from slate_amd.models.aux import allgather_dense as D

from dist_util import run_dist


def mk(kind, seed, m, n, nb=32, p=1, q=1, herm=False, dt=torch.float64):
    M = sl.HermitianMatrix(sl.Uplo.Lower, m, nb=nb, p=p, q=q, dtype=dt) if herm else \
        sl.Matrix(m, n, nb=nb, p=p, q=q, dtype=dt)
    M.insertLocalTiles()
    sl.generate_matrix(M, kind, seed)
    return M


def full(H):
    X = D(H)
    return torch.tril(X) + torch.tril(X, -1).mH


def check_mixed(p=1, q=1):
    n = 96
    A = mk("rand_dominant", 1, n, n, p=p, q=q)
    B = mk("rands", 2, n, 2, p=p, q=q)
    X = sl.Matrix(n, 2, nb=32, p=p, q=q)
    X.insertLocalTiles()
    A0, B0 = D(A).clone(), D(B).clone()
    info, it = sl.gesv_mixed(A, sl.Pivots(), B, X)
    assert info == 0 and it >= 0
    assert (A0 @ D(X) - B0).abs().max() < 1e-13
    H = mk("poev", 3, n, n, p=p, q=q, herm=True)
    Hf = full(H)
    info, it = sl.posv_mixed(H, B, X)
    assert info == 0 and (Hf @ D(X) - B0).abs().max() < 1e-13
    B1 = mk("rands", 4, n, 1, p=p, q=q)
    X1 = sl.Matrix(n, 1, nb=32, p=p, q=q)
    X1.insertLocalTiles()
    B1d = D(B1).clone()
    info, it = sl.gesv_mixed_gmres(A, sl.Pivots(), B1, X1)
    assert info == 0 and (A0 @ D(X1) - B1d).abs().max() < 1e-13
    info, it = sl.posv_mixed_gmres(H, B1, X1)
    assert info == 0 and (Hf @ D(X1) - B1d).abs().max() < 1e-13


def check_inverses(p=1, q=1):
    n = 80
    A = mk("rands", 5, n, n, p=p, q=q)
    A0 = D(A).clone()
    piv = sl.Pivots()
    assert sl.getrf(A, piv) == 0
    sl.getri(A, piv)
    assert (D(A) @ A0 - torch.eye(n, dtype=A0.dtype)).abs().max() < 1e-11
    H = mk("poev", 6, n, n, p=p, q=q, herm=True)
    Hf = full(H)
    assert sl.potrf(H) == 0
    assert sl.potri(H) == 0
    assert (full(H) @ Hf - torch.eye(n, dtype=Hf.dtype)).abs().max() < 1e-11
    T = mk("rands", 7, n, n, p=p, q=q)
    Td = torch.tril(D(T)) + n * torch.eye(n, dtype=torch.float64)
    sl.from_dense(T, Td)
    L = sl.TriangularMatrix(sl.Uplo.Lower, T)
    assert sl.trtri(L) == 0
    assert (torch.tril(D(T)) @ Td - torch.eye(n, dtype=Td.dtype)).abs().max() < 1e-12


def check_condest(p=1, q=1):
    n = 64
    A = mk("rands", 8, n, n, p=p, q=q)
    Ad = D(A).clone()
    anorm = float(sl.norm(sl.Norm.One, A))
    piv = sl.Pivots()
    sl.getrf(A, piv)
    rc = sl.gecondest(sl.Norm.One, A, piv, anorm)
    ref = 1 / (torch.linalg.norm(Ad, 1) * torch.linalg.norm(torch.linalg.inv(Ad), 1)).item()
    assert ref / 3 <= rc <= 3 * ref


def test_mixed():
    check_mixed()


def test_rbt():
    n = 128
    A = mk("rands", 9, n, n)
    B = mk("rands", 10, n, 3)
    A0, B0 = D(A).clone(), D(B).clone()
    assert sl.gesv_rbt(A, B) == 0
    assert (A0 @ D(B) - B0).abs().max() < 1e-11


@pytest.mark.parametrize("dt", [torch.float64, torch.complex128, torch.float32])
@pytest.mark.parametrize("depth", [1, 2, 3])
def test_butterfly_op_vs_dense(dt, depth):
    """ops.butterfly (all levels in one pass) against the explicit dense
    W = W_depth ... W_1, on rows and on the column index, W and W^T."""
    from slate_amd import ops
    from slate_amd.models.mixed import _butterfly_diag
    n, m = 48, 20
    dg = _butterfly_diag(n, depth, 3)
    W = torch.eye(n, dtype=torch.float64)
    for lvl in range(depth):
        size = n >> lvl
        h = size // 2
        Wl = torch.zeros(n, n, dtype=torch.float64)
        for o in range(0, n, size):
            for i in range(h):
                r0, r1 = dg[lvl, o + i], dg[lvl, o + h + i]
                Wl[o + i, o + i], Wl[o + i, o + h + i] = r0, r1
                Wl[o + h + i, o + i], Wl[o + h + i, o + h + i] = r0, -r1
        W = (Wl / 2 ** 0.5) @ W
    W = W.to(dt)
    g = torch.Generator().manual_seed(1)
    X = torch.randn(n, m, generator=g, dtype=torch.float64).to(dt).t().contiguous().t()
    Y = torch.randn(m, n, generator=g, dtype=torch.float64).to(dt).t().contiguous().t()
    rdt = torch.float32 if dt in (torch.float32, torch.complex64) else torch.float64
    tol = 1e-5 if rdt == torch.float32 else 1e-13
    for trans in (False, True):
        opW = W.mT if trans else W
        assert (ops.butterfly(X.clone(), dg.to(rdt), depth, trans, 'L') - opW @ X).abs().max() < tol
        assert (ops.butterfly(Y.clone(), dg.to(rdt), depth, trans, 'R') - Y @ opW.mT).abs().max() < tol


def _rbt_grid(rank, size, p, q):
    for n, nb in ((100, 16), (128, 16), (37, 8)):
        A = sl.Matrix(n, n, nb=nb, p=p, q=q)
        A.insertLocalTiles()
        sl.generate_matrix(A, "rands", 9)
        B = sl.Matrix(n, 3, nb=nb, p=p, q=q)
        B.insertLocalTiles()
        sl.generate_matrix(B, "rands", 10)
        A0, B0 = D(A).clone(), D(B).clone()
        assert sl.gesv_rbt(A, B, {Option.Depth: 2}) == 0
        assert (A0 @ D(B) - B0).abs().max() < 1e-11 * n


@pytest.mark.parametrize("grid", [(1, 1), (2, 2), (1, 3), (2, 1)], ids=lambda g: f"{g[0]}x{g[1]}")
def test_rbt_grid(grid):
    """RBT on the grid with padding (n not a multiple of the unit): every
    butterfly is local, no partial-pivoting fallback."""
    if grid == (1, 1):
        _rbt_grid(0, 1, 1, 1)
    else:
        run_dist(_rbt_grid, grid[0] * grid[1], *grid)


def test_inverses():
    check_inverses()


def test_condest():
    check_condest()


def _dist(rank, size, p, q):
    check_mixed(p, q)
    check_inverses(p, q)
    check_condest(p, q)


@pytest.mark.parametrize("grid", [(2, 1), (1, 2)])
def test_solvers_distributed(grid):
    run_dist(_dist, 2, *grid)


def _potri_both_uplo(rank, size, p, q):
    """potri / trtri / trtrm on the grid (distributed trsm/trmm, no gather):
    inverse correct for both storage triangles, the other triangle untouched."""
    from slate_amd.core.enums import Uplo
    for uplo in (Uplo.Lower, Uplo.Upper):
        n, nb = 70, 16
        A = sl.HermitianMatrix(uplo, n, nb=nb, p=p, q=q)
        A.insertLocalTiles()
        sl.generate_matrix(A, "poev", 3)
        X = D(A)
        lo = uplo == Uplo.Lower
        Af = (torch.tril(X) + torch.tril(X, -1).mT) if lo else (torch.triu(X) + torch.triu(X, 1).mT)
        other = (torch.triu(X, 1) if lo else torch.tril(X, -1)).clone()
        assert sl.potrf(A) == 0 and sl.potri(A) == 0
        Y = D(A)
        Yi = (torch.tril(Y) + torch.tril(Y, -1).mT) if lo else (torch.triu(Y) + torch.triu(Y, 1).mT)
        assert (Yi @ Af - torch.eye(n, dtype=Af.dtype)).abs().max().item() < 1e-10
        assert torch.equal(torch.triu(Y, 1) if lo else torch.tril(Y, -1), other)


@pytest.mark.parametrize("grid", [(1, 1), (2, 1), (1, 2), (2, 2)], ids=lambda g: f"{g[0]}x{g[1]}")
def test_potri_distributed(grid):
    if grid == (1, 1):
        _potri_both_uplo(0, 1, 1, 1)
    else:
        run_dist(_potri_both_uplo, grid[0] * grid[1], *grid)
