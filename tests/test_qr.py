"""QR / LQ / least-squares drivers (reference test strategy: test/test_geqrf.cc,
test_unmqr.cc, test_gelqf.cc, test_gels.cc -- residual checks
||A - QR|| / (||A|| n eps), ||Q^H Q - I||)."""
import pytest
import torch

import slate_amd as sl
from slate_amd.core.enums import Op, Option, Side, MethodGels
from slate_amd.core.matrix import TriangularFactors
from slate_amd.models import qr
from slate_amd.models.aux import allgather_dense as D

from dist_util import run_dist

DTYPES = [torch.float64, torch.complex128, torch.float32]


def _tol(dt):
    return 1e-4 if dt in (torch.float32, torch.complex64) else 1e-12


def _mat(m, n, nb, dt, seed, p=1, q=1, device=None):
    A = sl.Matrix(m, n, nb=nb, p=p, q=q, dtype=dt, device=device)
    A.insertLocalTiles(device=-1 if device is None or str(device) == "cpu" else 0)
    sl.generate_matrix(A, "rands", seed)
    return A


def _check_qr(m, n, nb, dt, p=1, q=1, device=None):
    A = _mat(m, n, nb, dt, 3, p, q, device)
    A0 = D(A).clone()
    T = TriangularFactors()
    qr.geqrf(A, T)
    F = D(A)
    k = min(m, n)
    R = torch.triu(F)[:k]
    Q = sl.Matrix(m, m, nb=nb, p=p, q=q, dtype=dt, device=device)
    Q.insertLocalTiles(device=-1 if device is None else 0)
    sl.set(0.0, 1.0, Q)
    qr.unmqr(Side.Left, Op.NoTrans, A, T, Q)
    Qd = D(Q)
    scale = max(1.0, A0.abs().max().item()) * max(m, n)
    assert (Qd[:, :k] @ R - A0).abs().max().item() / scale < _tol(dt)
    assert (Qd.conj().T @ Qd - torch.eye(m, dtype=dt, device=Qd.device)).abs().max().item() / m < _tol(dt)
    return A, T, Qd


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("mn", [(300, 200, 64), (128, 128, 32), (96, 160, 32), (30, 40, 16)])
def test_geqrf_unmqr(dt, mn):
    m, n, nb = mn
    _check_qr(m, n, nb, dt)


@pytest.mark.parametrize("side", [Side.Left, Side.Right])
@pytest.mark.parametrize("op", [Op.NoTrans, Op.ConjTrans])
def test_unmqr_variants(side, op):
    dt = torch.complex128
    m, n, nb = 160, 96, 32
    A, T, Qd = _check_qr(m, n, nb, dt)
    Cshape = (m, 40) if side == Side.Left else (40, m)
    C = _mat(*Cshape, nb, dt, 9)
    C0 = D(C).clone()
    qr.unmqr(side, op, A, T, C)
    Qo = Qd if op == Op.NoTrans else Qd.conj().T
    ref = Qo @ C0 if side == Side.Left else C0 @ Qo
    assert (D(C) - ref).abs().max().item() < 1e-12


@pytest.mark.parametrize("dt", [torch.float64, torch.complex128])
def test_gelqf_unmlq(dt):
    m, n, nb = 96, 160, 32
    A = _mat(m, n, nb, dt, 4)
    A0 = D(A).clone()
    T = TriangularFactors()
    qr.gelqf(A, T)
    L = torch.tril(D(A))[:, :m]
    Q = _mat(n, n, nb, dt, 1)
    sl.set(0.0, 1.0, Q)
    qr.unmlq(Side.Left, Op.NoTrans, A, T, Q)
    Qd = D(Q)
    # A = L Q[:m, :]
    assert (L @ Qd[:m] - A0).abs().max().item() < 1e-12 * n


@pytest.mark.parametrize("dt", [torch.float64, torch.complex128])
@pytest.mark.parametrize("shape", [(200, 80), (80, 200)])
def test_gels(dt, shape):
    m, n = shape
    nb, nrhs = 32, 5
    A = _mat(m, n, nb, dt, 5)
    A0 = D(A).clone()
    BX = _mat(max(m, n), nrhs, nb, dt, 6)
    B0 = D(BX)[:m].clone()
    qr.gels(A, TriangularFactors(), BX)
    X = D(BX)[:n]
    Xref = torch.linalg.lstsq(A0, B0).solution if m >= n else torch.linalg.pinv(A0) @ B0
    assert (X - Xref).abs().max().item() < 1e-10


def test_gels_cholqr():
    m, n, nb, nrhs = 300, 60, 32, 3
    dt = torch.float64
    A = _mat(m, n, nb, dt, 7)
    A0 = D(A).clone()
    BX = _mat(m, nrhs, nb, dt, 8)
    B0 = D(BX).clone()
    qr.gels(A, TriangularFactors(), BX, {Option.MethodGels: MethodGels.CholQR})
    X = D(BX)[:n]
    Xref = torch.linalg.lstsq(A0, B0).solution
    assert (X - Xref).abs().max().item() < 1e-9


def test_cholqr():
    m, n, nb = 256, 64, 32
    dt = torch.float64
    A = _mat(m, n, nb, dt, 11)
    A0 = D(A).clone()
    R = _mat(n, n, nb, dt, 1)
    assert qr.cholqr(A, R) == 0
    Qd, Rd = D(A), torch.triu(D(R))
    assert (Qd @ Rd - A0).abs().max().item() < 1e-12 * m
    assert (Qd.T @ Qd - torch.eye(n, dtype=dt)).abs().max().item() < 1e-10


# ---------------------------------------------------------------- distributed
def _dist_qr(rank, size, p, q):
    for dt in (torch.float64, torch.complex128):
        _check_qr(150, 100, 32, dt, p, q)
        # least squares on the grid
        A = _mat(150, 60, 32, dt, 5, p, q)
        A0 = D(A).clone()
        BX = _mat(150, 3, 32, dt, 6, p, q)
        B0 = D(BX).clone()
        qr.gels(A, TriangularFactors(), BX)
        X = D(BX)[:60]
        assert (X - torch.linalg.lstsq(A0, B0).solution).abs().max().item() < 1e-10


@pytest.mark.parametrize("grid", [(2, 1), (1, 2), (2, 2), (4, 1)], ids=lambda g: f"{g[0]}x{g[1]}")
def test_qr_distributed(grid):
    run_dist(_dist_qr, grid[0] * grid[1], *grid)


def _dist_qr_la(rank, size, p, q):
    """TSQR with lookahead 0..2, ragged last tiles and ranks without rows."""
    for (m, n, nb, la) in [(200, 120, 16, 0), (333, 90, 32, 2), (96, 96, 16, 1), (70, 100, 16, 1)]:
        A = _mat(m, n, nb, torch.float64, 12, p, q)
        A0 = D(A).clone()
        T = TriangularFactors()
        qr.geqrf(A, T, {Option.Lookahead: la})
        R = torch.triu(D(A))[:n]
        assert (R.T @ R - A0.T @ A0).abs().max().item() / (A0.abs().max().item() ** 2 * m) < 1e-13
        C = _mat(m, 7, nb, torch.float64, 13, p, q)
        C0 = D(C).clone()
        qr.unmqr(Side.Left, Op.ConjTrans, A, T, C)
        qr.unmqr(Side.Left, Op.NoTrans, A, T, C)
        assert (D(C) - C0).abs().max().item() < 1e-12


@pytest.mark.parametrize("grid", [(4, 1), (2, 2)], ids=lambda g: f"{g[0]}x{g[1]}")
def test_tsqr_lookahead(grid):
    run_dist(_dist_qr_la, grid[0] * grid[1], *grid)


# ---------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float64, torch.complex128, torch.float32])
@pytest.mark.parametrize("mn", [(1000, 256), (4096, 512), (300, 300), (64, 200)])
def test_geqrf_panel_gpu(dt, mn):
    from slate_amd import ops
    m, n = mn
    dev = torch.device("cuda")
    A0 = torch.randn(m, n, dtype=dt, device=dev)
    A = A0.t().contiguous().t()
    k = min(m, n)
    tau = torch.zeros(k, dtype=dt, device=dev)
    T, V = ops.geqrf(A, tau)
    torch.cuda.synchronize()
    Q = torch.eye(m, dtype=dt, device=dev) - V @ T @ V.conj().T
    R = torch.triu(A)[:k]
    tol = 1e-3 if dt == torch.float32 else 1e-11
    assert ((Q[:, :k] @ R - A0).abs().max() / A0.abs().max()).item() < tol
    assert (Q.conj().T @ Q - torch.eye(m, dtype=dt, device=dev)).abs().max().item() < tol


@pytest.mark.gpu
def test_geqrf_gpu_driver():
    _check_qr(1500, 1000, 256, torch.float64, device=torch.device("cuda"))


def _panel_checks(A0, A, tau, T, V):
    """Q = I - V T V^T without forming it: Q [R; 0] = A0, and Q^T Q = I
    (<=> T^T (V^T V) T = T + T^T, V unit lower hence full rank)."""
    b = A.shape[1]
    R = torch.triu(A)[:b]
    QR = -(V @ (T @ (V[:b].t() @ R)))
    QR[:b] += R
    assert ((QR - A0).abs().max() / A0.abs().max()).item() < 1e-12
    O = T.t() @ (V.t() @ V) @ T - T - T.t()
    assert O.abs().max().item() < 1e-11
    assert torch.equal(torch.diagonal(T), tau)
    assert torch.equal(torch.triu(V[:b]), torch.eye(b, dtype=A.dtype, device=A.device))
    assert torch.equal(torch.tril(A, -1), torch.tril(V, -1))


@pytest.mark.gpu
@pytest.mark.parametrize("mb", [(16384, 256), (8192, 128), (65536, 256), (3000, 200), (1024, 16)])
def test_geqrf_cholqr_panel(mb):
    """Tall fp64 panels (m >= 8 b, b <= 256) take the shifted CholeskyQR3 +
    Householder reconstruction path (csrc/hip/qr_fast.hip); the output has
    the Householder panel's form (R, unit-lower V, tau = diag(T), T)."""
    from slate_amd import ops
    m, b = mb
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(m + b)
    A0 = torch.randn(m, b, dtype=torch.float64, generator=g).to(dev)
    A0[:, 1] *= 1e5                      # unequal column scales
    A = A0.t().contiguous().t()
    tau = torch.zeros(b, dtype=torch.float64, device=dev)
    T, V = ops.geqrf(A, tau)
    torch.cuda.synchronize()
    _panel_checks(A0, A, tau, T, V)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["zero_dup", "rank10", "graded"])
def test_geqrf_cholqr_breakdown_falls_back(kind):
    """Panels that break CholeskyQR2 down (rank-deficient, or kappa beyond
    u^-1/2): decided on the device without a host read-back, the panel is
    restored, perturbed by 10 u ||A|| and factored by the gated shifted
    CholeskyQR3 with a pivot floor (csrc/hip/qr_fast.hip); the result must
    still be a backward-stable QR with orthonormal Q."""
    from slate_amd import ops
    m, b = 8192, 64
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(3)
    A0 = torch.randn(m, b, dtype=torch.float64, generator=g)
    if kind == "zero_dup":
        A0[:, 10] = 0.0
        A0[:, 20] = A0[:, 3]
    elif kind == "rank10":
        A0 = torch.randn(m, 10, dtype=torch.float64, generator=g) @ torch.randn(10, b, dtype=torch.float64,
                                                                                  generator=g)
    else:
        A0 = A0 * torch.logspace(0, -13, b, dtype=torch.float64)
    A0 = A0.to(dev)
    A = A0.t().contiguous().t()
    tau = torch.zeros(b, dtype=torch.float64, device=dev)
    T, V = ops.geqrf(A, tau)
    torch.cuda.synchronize()
    _panel_checks(A0, A, tau, T, V)


@pytest.mark.gpu
def test_geqrf_gpu_driver_tall():
    """Tall matrix: every panel takes the CholeskyQR path."""
    _check_qr(8192, 512, 128, torch.float64, device=torch.device("cuda"))


@pytest.mark.parametrize("dt", [torch.float64, torch.complex128])
@pytest.mark.parametrize("mn", [(300, 200, 32), (512, 256, 32), (200, 300, 32)])
def test_geqrf_grouped_bulk_update(dt, mn, monkeypatch):
    """Bulk trailing updates of two panels applied as one merged block
    reflector (SLATE_AMD_QR_GROUP=2, the GPU default on one process column)
    give the same factorization as per-panel updates."""
    monkeypatch.setenv("SLATE_AMD_QR_GROUP", "2")
    m, n, nb = mn
    _check_qr(m, n, nb, dt)
