"""RowMajor (transposed-storage) LU on the GPU (models/lu.py _getrf_p1 with
T): interchanges move contiguous columns of T = A^T (laswp_cols), the
trailing update is an NT GEMM.  Checked against an fp64 torch reference of
P A = L U, against the column-major path, and the explicit-L11-inverse
growth guard: a step whose inverse grows past the limit makes
the driver redo the factorization with the trsm form."""
import pytest
import torch

import slate_amd as sl
from slate_amd import ops
from slate_amd.models import lu as lu_mod

pytestmark = pytest.mark.gpu


def _lu_residual(F0, F, ipiv):
    m, n = F0.shape
    k = min(m, n)
    L = torch.tril(F[:, :k], -1) + torch.eye(m, k, dtype=F.dtype, device=F.device)
    U = torch.triu(F[:k, :])
    perm = list(range(m))
    for i, j in enumerate(ipiv.tolist()):
        perm[i], perm[j] = perm[j], perm[i]
    PA = F0[torch.as_tensor(perm, device=F.device)]
    return ((L @ U - PA).norm() / F0.norm()).item()


def test_laswp_cols_matches_laswp():
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(3)
    m, n = 3000, 700
    A = torch.randn(m, n, dtype=torch.float64, generator=g).to(dev).mT.contiguous().mT
    ipiv = torch.tensor([min(m - 1, i + int(x)) for i, x in enumerate(torch.randint(0, 900, (600,), generator=g))],
                        dtype=torch.int64, device=dev)
    B = A.clone()
    ops.laswp(B, ipiv, 0, 600)                     # rows of A
    T = ops.as_colmajor(A.t())                     # n x m column-major = A^T
    ops.laswp_cols(T, ipiv, 0, 600)                # columns of A^T
    assert torch.equal(T.t(), B)
    # backward (incx = -1) undoes it
    ops.laswp_cols(T, ipiv, 0, 600, incx=-1)
    assert torch.equal(T.t(), A)


@pytest.mark.parametrize("mn,nb,la", [((2048, 2048), 256, 2), ((1800, 1800), 256, 1),
                                      ((3000, 1200), 256, 2), ((1000, 2600), 256, 1)])
def test_getrf_rowmajor_matches_reference(mn, nb, la, monkeypatch):
    m, n = mn
    dev = torch.device("cuda")
    res = {}
    for rm in ("1", "0"):
        monkeypatch.setenv("SLATE_AMD_LU_ROWMAJOR", rm)
        A = sl.Matrix(m, n, nb=nb, device=dev)
        A.insertLocalTiles(device=dev)
        sl.generate_matrix(A, "rands", seed=7)
        F0 = A.storage.local[A.storage.origin_slot][:m, :n].clone()
        piv = sl.Pivots()
        assert sl.getrf(A, piv, {sl.Option.Lookahead: la}) == 0
        F = A.storage.local[A.storage.origin_slot][:m, :n]
        res[rm] = _lu_residual(F0, F, piv.ipiv[:min(m, n)])
    assert res["1"] < 1e-13 and res["0"] < 1e-13, res


def test_getrf_rowmajor_inverse_growth_redo(monkeypatch):
    """Force the growth limit below any inverse: the driver must notice at
    the end, redo the factorization with trsm, and still be exact."""
    monkeypatch.setenv("SLATE_AMD_LU_INV_MIN", "256")
    monkeypatch.setenv("SLATE_AMD_LU_INV_GROWTH", "0.5")
    dev = torch.device("cuda")
    n, nb = 2048, 256
    A = sl.Matrix(n, n, nb=nb, device=dev)
    A.insertLocalTiles(device=dev)
    sl.generate_matrix(A, "rands", seed=8)
    F0 = A.storage.local[A.storage.origin_slot][:n, :n].clone()
    lu_mod.LU_INV_REDO.clear()
    piv = sl.Pivots()
    assert sl.getrf(A, piv, {sl.Option.Lookahead: 1}) == 0
    assert lu_mod.LU_INV_REDO, "growth guard did not fire"
    assert _lu_residual(F0, A.storage.local[A.storage.origin_slot][:n, :n], piv.ipiv[:n]) < 1e-13


def test_getrf_wilkinson_like_growth_guarded(monkeypatch):
    """A matrix whose L11 inverse grows like 2^(k-1): every multiplier of
    the first panel is -1 (the lower part of Wilkinson's growth matrix), so
    |L11^{-1}| reaches 2^(nb-2).  With the default guard the result keeps
    the backward error of the trsm form."""
    monkeypatch.setenv("SLATE_AMD_LU_INV_MIN", "256")
    dev = torch.device("cuda")
    n, nb = 1024, 256
    # first panel: unit diagonal, -1 below it (no interchanges: ties keep
    # the upper row), zero A12; the rest a well-conditioned block
    W = torch.eye(n, dtype=torch.float64)
    W[:, :nb] -= torch.tril(torch.ones(n, nb, dtype=torch.float64), -1)
    W[nb:, nb:] += 0.01 * torch.randn(n - nb, n - nb, dtype=torch.float64,
                                      generator=torch.Generator().manual_seed(5))
    A = sl.Matrix(n, n, nb=nb, device=dev)
    A.insertLocalTiles(device=dev)
    A.storage.local[A.storage.origin_slot][:n, :n].copy_(W.to(dev))
    lu_mod.LU_INV_REDO.clear()
    piv = sl.Pivots()
    sl.getrf(A, piv, {sl.Option.Lookahead: 1})
    r_guarded = _lu_residual(W.to(dev), A.storage.local[A.storage.origin_slot][:n, :n], piv.ipiv[:n])
    assert lu_mod.LU_INV_REDO, "the inverse of this L11 grows like 2^(nb-2): the guard must fire"
    monkeypatch.setenv("SLATE_AMD_LU_INV_MIN", "0")
    A2 = sl.Matrix(n, n, nb=nb, device=dev)
    A2.insertLocalTiles(device=dev)
    A2.storage.local[A2.storage.origin_slot][:n, :n].copy_(W.to(dev))
    piv2 = sl.Pivots()
    sl.getrf(A2, piv2, {sl.Option.Lookahead: 1})
    r_trsm = _lu_residual(W.to(dev), A2.storage.local[A2.storage.origin_slot][:n, :n], piv2.ipiv[:n])
    assert r_guarded <= 10 * r_trsm + 1e-15, (r_guarded, r_trsm)
