"""Norms of matrices whose storage has no 2-D block-cyclic map (LAPACK-wrapped
arrays on a p x q grid): the gathered op(A) goes through the genorm kernels
with the stored triangle masked inside the kernel (models/aux.py
_dense_norm).  Checked against torch fp64 on the explicit full matrix for
general / trapezoid (unit and non-unit) / symmetric / Hermitian, all four
norms, NoTrans and ConjTrans views."""
import pytest
import torch

import slate_amd as sl
from slate_amd.core.enums import Diag, Op, Uplo

from dist_util import run_dist


def _ref(F, nt):
    a = F.abs()
    return {"max": a.max(), "one": a.sum(0).max(), "inf": a.sum(1).max(), "fro": torch.sqrt((a * a).sum())}[nt]


def _full(X, kind, uplo, unit=False):
    L = torch.tril(X) if uplo == Uplo.Lower else torch.triu(X)
    if kind == "trapezoid":
        if unit:
            L = L.clone()
            L.diagonal().fill_(1)
        return L
    if kind == "symmetric":
        return L + L.transpose(0, 1) - torch.diag(torch.diagonal(L))
    H = L + L.mH
    H.diagonal().copy_(torch.diagonal(L).real.to(X.dtype))
    return H


def _cm(X):
    return X.t().contiguous().t()


def _check(rank, size):
    torch.manual_seed(5)
    m, n, nb = 37, 29, 8
    for dt in (torch.float64, torch.complex128):
        G = torch.randn(m, n, dtype=dt)
        A = sl.Matrix.fromLAPACK(m, n, _cm(G), nb=nb, p=2, q=1)
        assert A.storage.bc is None
        S = torch.randn(n, n, dtype=dt)
        for nt in ("max", "one", "inf", "fro"):
            got = sl.norm(nt, A)
            assert abs(got - float(_ref(G, nt))) <= 1e-12 * float(_ref(G, nt)), (dt, nt, "general")
            got = sl.norm(nt, A.conj_transpose())
            assert abs(got - float(_ref(G.mH, nt))) <= 1e-12 * float(_ref(G, "fro")), (dt, nt, "general^H")
            for uplo in (Uplo.Lower, Uplo.Upper):
                for unit in (False, True):
                    T = sl.TrapezoidMatrix.fromLAPACK(uplo, m, n, _cm(G), nb=nb, p=2, q=1,
                                                      diag=Diag.Unit if unit else Diag.NonUnit)
                    F = _full(G, "trapezoid", uplo, unit)
                    got = sl.norm(nt, T)
                    assert abs(got - float(_ref(F, nt))) <= 1e-12 * float(_ref(F, "fro")), (dt, nt, uplo, unit)
                H = sl.HermitianMatrix.fromLAPACK(uplo, n, _cm(S), nb=nb, p=2, q=1)
                F = _full(S, "hermitian", uplo)
                got = sl.norm(nt, H)
                assert abs(got - float(_ref(F, nt))) <= 1e-12 * float(_ref(F, "fro")), (dt, nt, uplo, "herm")
                Y = sl.SymmetricMatrix.fromLAPACK(uplo, n, _cm(S), nb=nb, p=2, q=1)
                F = _full(S, "symmetric", uplo)
                got = sl.norm(nt, Y)
                assert abs(got - float(_ref(F, nt))) <= 1e-12 * float(_ref(F, "fro")), (dt, nt, uplo, "sym")
    G = torch.randn(m, n, dtype=torch.float64)
    G[3, 4] = float("nan")
    A = sl.Matrix.fromLAPACK(m, n, _cm(G), nb=nb, p=2, q=1)
    assert sl.norm("max", A) != sl.norm("max", A)


def test_dense_norm_without_block_cyclic_map():
    run_dist(_check, 2)


def test_dense_norm_views_match_op():
    X = torch.randn(6, 4, dtype=torch.float64)
    F = X.clone()
    assert float(_ref(F.T, "one")) == pytest.approx(float(_ref(F, "inf")))
    assert Op.NoTrans != Op.Trans
