"""Triangle-pentagonal QR/LQ tile kernels (tpqrt/tpmqrt/tplqt/tpmlqt) against
an fp64 PyTorch reference of the same ops (reference tester:
test/test_tpqrt.cc -- ||Q^H [A; B] - [R; 0]|| and ||I - Q^H Q||)."""
import pytest
import torch

from slate_amd import ops

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _dev(d):
    if d == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device(d)


def _cm(x):
    return ops.as_colmajor(x.t().contiguous().t())


def _pentagon(m, n, l, dt, g):
    B = torch.randn(m, n, dtype=dt, generator=g)
    for c in range(n):
        rows = min(m, m - l + min(l, c + 1))
        B[rows:, c] = 0
    return B


def _q(V, T):
    m, n = V.shape
    Vf = torch.cat([torch.eye(n, dtype=V.dtype), V], 0)
    return torch.eye(n + m, dtype=V.dtype) - Vf @ T @ Vf.mH


@pytest.mark.parametrize("dev", DEVICES)
@pytest.mark.parametrize("dt", [torch.float64, torch.complex128])
@pytest.mark.parametrize("m,n,l,ib", [(40, 24, 0, 8), (24, 24, 24, 8), (50, 30, 17, 16), (12, 40, 12, 32),
                                      (200, 96, 96, 32), (7, 5, 3, 64)])
def test_tpqrt(dev, dt, m, n, l, ib):
    d = _dev(dev)
    g = torch.Generator().manual_seed(m * 100 + n + l)
    A0 = torch.triu(torch.randn(n, n, dtype=dt, generator=g))
    B0 = _pentagon(m, n, l, dt, g)
    A, B = _cm(A0.clone()).to(d), _cm(B0.clone()).to(d)
    A, B = _cm(A), _cm(B)
    T, V, tau = ops.tpqrt(l, A, B, ib=ib)
    T, V, A, B = T.cpu(), V.cpu(), A.cpu(), B.cpu()
    R = torch.triu(A)
    Q = _q(V, T)
    S0 = torch.cat([A0, B0], 0)
    eps = torch.finfo(torch.float64).eps
    nrm = S0.norm()
    # orthogonality, backward error, zero-pattern of V, R in place
    assert (Q.mH @ Q - torch.eye(n + m, dtype=dt)).norm() < 50 * eps * (n + m)
    QhS = Q.mH @ S0
    assert (QhS[:n] - R).norm() / nrm < 50 * eps * (n + m)
    assert QhS[n:].norm() / nrm < 50 * eps * (n + m)
    for c in range(n):
        rows = min(m, m - l + min(l, c + 1))
        assert V[rows:, c].abs().sum().item() == 0
    assert torch.equal(V, B)                 # reflectors in place of the pentagon
    # |diag R| equals the reference QR's
    Rr = torch.linalg.qr(S0, mode="r")[1]
    k = min(n, n + m)
    assert torch.allclose(R.diagonal()[:k].abs(), Rr.diagonal()[:k].abs(), rtol=1e-10, atol=1e-10 * nrm.item())


@pytest.mark.parametrize("dev", DEVICES)
@pytest.mark.parametrize("dt", [torch.float64, torch.complex128])
@pytest.mark.parametrize("side,trans", [("L", "C"), ("L", "N"), ("R", "N"), ("R", "C")])
def test_tpmqrt(dev, dt, side, trans):
    d = _dev(dev)
    g = torch.Generator().manual_seed(3)
    m, n, l, nc = 33, 20, 9, 13
    A0 = torch.triu(torch.randn(n, n, dtype=dt, generator=g))
    B0 = _pentagon(m, n, l, dt, g)
    A, B = _cm(A0.clone()).to(d), _cm(B0.clone()).to(d)
    T, V, tau = ops.tpqrt(l, A, B, ib=8)
    Q = _q(V.cpu(), T.cpu())
    opQ = Q if trans == "N" else Q.mH
    if side == "L":
        C1 = torch.randn(n, nc, dtype=dt, generator=g)
        C2 = torch.randn(m, nc, dtype=dt, generator=g)
        ref = opQ @ torch.cat([C1, C2], 0)
        X1, X2 = _cm(C1.clone()).to(d), _cm(C2.clone()).to(d)
        ops.tpmqrt(side, trans, V, T, X1, X2)
        got = torch.cat([X1.cpu(), X2.cpu()], 0)
    else:
        C1 = torch.randn(nc, n, dtype=dt, generator=g)
        C2 = torch.randn(nc, m, dtype=dt, generator=g)
        ref = torch.cat([C1, C2], 1) @ opQ
        X1, X2 = _cm(C1.clone()).to(d), _cm(C2.clone()).to(d)
        ops.tpmqrt(side, trans, V, T, X1, X2)
        got = torch.cat([X1.cpu(), X2.cpu()], 1)
    assert (got - ref).norm() / ref.norm() < 1e-13


@pytest.mark.parametrize("dev", DEVICES)
@pytest.mark.parametrize("dt", [torch.float64, torch.complex128])
def test_tplqt_tpmlqt(dev, dt):
    d = _dev(dev)
    g = torch.Generator().manual_seed(5)
    k, m, l = 18, 27, 10
    A0 = torch.tril(torch.randn(k, k, dtype=dt, generator=g))
    B0 = _pentagon(m, k, l, dt, g).mH.contiguous()          # k x m, last l columns lower trapezoidal
    A, B = _cm(A0.clone()).to(d), _cm(B0.clone()).to(d)
    T, W, tau = ops.tplqt(l, A, B, ib=8)
    L = torch.tril(A.cpu())
    # [A B] = [L 0] Q  ->  [A B] Q^H = [L 0]
    X1, X2 = _cm(A0.clone()).to(d), _cm(B0.clone()).to(d)
    ops.tpmlqt("R", "C", W, T, X1, X2)
    nrm = torch.cat([A0, B0], 1).norm()
    assert (X1.cpu() - L).norm() / nrm < 1e-13
    assert X2.cpu().norm() / nrm < 1e-13
