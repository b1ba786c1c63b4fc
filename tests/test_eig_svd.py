"""Eigenvalue / SVD drivers (reference: test/test_heev.cc, test_hegv.cc,
test_svd.cc, test_stedc*.cc -- residual ||A Z - Z Lambda|| / (||A|| n),
orthogonality ||Z^H Z - I|| / n, values vs. a sequential reference)."""
import pytest
import torch

import slate_amd as sl
from slate_amd.core.enums import MethodEig, Option, Uplo
from slate_amd import ops
from slate_amd.models import eig as E
from slate_amd.models import svd as S
from slate_amd.models.aux import allgather_dense as D

from dist_util import run_dist


def _herm(n, nb, dt, uplo, p=1, q=1, seed=3, device=None):
    A = sl.HermitianMatrix(uplo, n, nb=nb, p=p, q=q, dtype=dt, device=device)
    A.insertLocalTiles(device=-1 if device is None else 0)
    sl.generate_matrix(A, "rands", seed)
    return A


def _check_heev(n, nb, dt, uplo, method, p=1, q=1, device=None, ib=16):
    A = _herm(n, nb, dt, uplo, p, q, device=device)
    Af = E._dense_hermitian(A).cpu()
    Z = sl.Matrix(n, n, nb=nb, p=p, q=q, dtype=dt, device=device)
    Z.insertLocalTiles(device=-1 if device is None else 0)
    w = sl.heev(A, None, Z, {Option.InnerBlocking: ib, Option.MethodEig: method})
    Zd = D(Z).cpu()
    wr = torch.linalg.eigvalsh(Af)
    sc = max(1.0, Af.abs().max().item()) * n
    assert (w.cpu() - wr).abs().max().item() / sc < 1e-13
    assert (Af @ Zd - Zd * w.to(dt).cpu()).abs().max().item() / sc < 1e-13
    assert (Zd.mH @ Zd - torch.eye(n, dtype=dt)).abs().max().item() / n < 1e-13


@pytest.mark.parametrize("dt", [torch.float64, torch.complex128])
@pytest.mark.parametrize("uplo", [Uplo.Lower, Uplo.Upper])
@pytest.mark.parametrize("method", [MethodEig.DC, MethodEig.QR])
def test_heev(dt, uplo, method):
    _check_heev(130, 32, dt, uplo, method)


def test_heev_values_only():
    A = _herm(100, 32, torch.float64, Uplo.Lower)
    Af = E._dense_hermitian(A)
    w = sl.eig_vals(A)
    assert (w - torch.linalg.eigvalsh(Af)).abs().max().item() < 1e-12


def test_stedc_steqr_sterf():
    torch.manual_seed(1)
    n = 257
    d, e = torch.randn(n, dtype=torch.float64), torch.randn(n - 1, dtype=torch.float64)
    T = torch.diag(d) + torch.diag(e, 1) + torch.diag(e, -1)
    wr = torch.linalg.eigvalsh(T)
    assert (sl.sterf(d, e) - wr).abs().max() < 1e-12
    for w, Z in (sl.steqr(d, e), sl.stedc(d, e, leaf=16)):
        assert (w - wr).abs().max() < 1e-12
        assert (T @ Z - Z * w).abs().max() < 1e-12
        assert (Z.T @ Z - torch.eye(n, dtype=torch.float64)).abs().max() < 1e-12
    # clustered / repeated eigenvalues (deflation paths)
    d2 = torch.ones(n, dtype=torch.float64)
    d2[::3] = 2.0
    e2 = torch.full((n - 1,), 1e-9, dtype=torch.float64)
    T2 = torch.diag(d2) + torch.diag(e2, 1) + torch.diag(e2, -1)
    w, Z = sl.stedc(d2, e2, leaf=16)
    assert (T2 @ Z - Z * w).abs().max() < 1e-12
    assert (Z.T @ Z - torch.eye(n, dtype=torch.float64)).abs().max() < 1e-11


@pytest.mark.parametrize("itype", [1, 2, 3])
def test_hegv(itype):
    n, nb = 80, 16
    dt = torch.float64
    A = _herm(n, nb, dt, Uplo.Lower, seed=4)
    Bm = sl.HermitianMatrix(Uplo.Lower, n, nb=nb, dtype=dt)
    Bm.insertLocalTiles()
    sl.generate_matrix(Bm, "poev", 5)
    Af, Bf = E._dense_hermitian(A), E._dense_hermitian(Bm)
    Z = sl.Matrix(n, n, nb=nb, dtype=dt)
    Z.insertLocalTiles()
    w = sl.hegv(itype, A, Bm, None, Z, {Option.InnerBlocking: 16})
    X = D(Z)
    if itype == 1:
        R = Af @ X - Bf @ X * w
    elif itype == 2:
        R = Af @ Bf @ X - X * w
    else:
        R = Bf @ Af @ X - X * w
    assert R.abs().max().item() / (Af.abs().max() * Bf.abs().max() * n).item() < 1e-12


@pytest.mark.parametrize("dt", [torch.float64, torch.complex128])
@pytest.mark.parametrize("shape", [(120, 80), (80, 120), (64, 64)])
def test_svd(dt, shape):
    m, n = shape
    k = min(m, n)
    A = sl.Matrix(m, n, nb=32, dtype=dt)
    A.insertLocalTiles()
    sl.generate_matrix(A, "rands", 3)
    Ad = D(A).clone()
    U = sl.Matrix(m, k, nb=32, dtype=dt)
    U.insertLocalTiles()
    VH = sl.Matrix(k, n, nb=32, dtype=dt)
    VH.insertLocalTiles()
    s = sl.svd(A, None, U, VH, {Option.InnerBlocking: 16})
    Ud, Vd = D(U), D(VH)
    assert (s - torch.linalg.svdvals(Ad)).abs().max().item() < 1e-12
    assert (Ud @ torch.diag(s.to(dt)) @ Vd - Ad).abs().max().item() < 1e-12
    assert (Ud.mH @ Ud - torch.eye(k, dtype=dt)).abs().max().item() < 1e-12
    assert (Vd @ Vd.mH - torch.eye(k, dtype=dt)).abs().max().item() < 1e-12


def test_svd_vals_bdsqr():
    torch.manual_seed(2)
    n = 200
    d, e = torch.randn(n, dtype=torch.float64), torch.randn(n - 1, dtype=torch.float64)
    B = torch.diag(d) + torch.diag(e, 1)
    s, U, VT = sl.bdsqr(d, e)
    assert (s - torch.linalg.svdvals(B)).abs().max() < 1e-12
    assert (U @ torch.diag(s) @ VT - B).abs().max() < 1e-12


def _dist_eig(rank, size, p, q):
    from slate_amd.models import eig_dist
    eig_dist.BCAST_STATS.update(host_bytes=0, host_max=0, dev_bytes=0)
    _check_heev(90, 16, torch.float64, Uplo.Lower, MethodEig.DC, p, q)
    st = dict(eig_dist.BCAST_STATS)
    # stage-2 reflectors (~n^2/2 words) go on the device path; the host path
    # carries only O(n) vectors (d, e, count)
    assert st["host_max"] <= 8 * 90, st
    assert st["dev_bytes"] >= 8 * 90 * 16, st
    A = sl.Matrix(70, 50, nb=16, p=p, q=q)
    A.insertLocalTiles()
    sl.generate_matrix(A, "rands", 9)
    Ad = D(A).clone()
    U = sl.Matrix(70, 50, nb=16, p=p, q=q)
    U.insertLocalTiles()
    VH = sl.Matrix(50, 50, nb=16, p=p, q=q)
    VH.insertLocalTiles()
    s = sl.svd(A, None, U, VH, {Option.InnerBlocking: 8})
    assert (D(U) @ torch.diag(s) @ D(VH) - Ad).abs().max().item() < 1e-12


@pytest.mark.parametrize("grid", [(2, 1), (1, 2)])
def test_eig_svd_distributed(grid):
    run_dist(_dist_eig, 2, *grid)


def _dist_heev_only(rank, size, p, q):
    for dt, uplo in ((torch.float64, Uplo.Lower), (torch.complex128, Uplo.Upper)):
        _check_heev(100, 16, dt, uplo, MethodEig.DC, p, q)
    _check_heev(77, 16, torch.float64, Uplo.Lower, MethodEig.QR, p, q)
    # generalized problem: distributed hegst (trsm/trmm on a full copy)
    n, nb = 64, 16
    A = _herm(n, nb, torch.float64, Uplo.Lower, p, q, seed=4)
    Bm = sl.HermitianMatrix(Uplo.Lower, n, nb=nb, p=p, q=q)
    Bm.insertLocalTiles()
    sl.generate_matrix(Bm, "poev", 5)
    Af, Bf = E._dense_hermitian(A), E._dense_hermitian(Bm)
    Z = sl.Matrix(n, n, nb=nb, p=p, q=q)
    Z.insertLocalTiles()
    w = sl.hegv(1, A, Bm, None, Z)
    X = D(Z)
    assert (Af @ X - Bf @ X * w).abs().max().item() / (Af.abs().max() * Bf.abs().max() * n).item() < 1e-12


@pytest.mark.parametrize("grid", [(2, 2), (4, 1), (1, 3)], ids=lambda g: f"{g[0]}x{g[1]}")
def test_heev_grid(grid):
    """he2hb on the process grid (no dense gather), band to rank 0, grid back-transforms."""
    run_dist(_dist_heev_only, grid[0] * grid[1], *grid)


def test_heev_dist_path_one_rank(monkeypatch):
    monkeypatch.setenv("SLATE_AMD_EIG_DIST", "1")
    _check_heev(100, 16, torch.float64, Uplo.Lower, MethodEig.DC)
    _check_heev(64, 16, torch.complex128, Uplo.Upper, MethodEig.QR)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float64, torch.complex128])
def test_heev_gpu(dt):
    _check_heev(600, 128, dt, Uplo.Lower, MethodEig.DC, device=torch.device("cuda"), ib=64)


@pytest.mark.gpu
def test_svd_gpu():
    dev = torch.device("cuda")
    m, n = 500, 300
    A = sl.Matrix(m, n, nb=128, dtype=torch.float64, device=dev)
    A.insertLocalTiles(device=0)
    sl.generate_matrix(A, "rands", 3)
    Ad = D(A).clone()
    U = sl.Matrix(m, n, nb=128, device=dev)
    U.insertLocalTiles(device=0)
    VH = sl.Matrix(n, n, nb=128, device=dev)
    VH.insertLocalTiles(device=0)
    s = sl.svd(A, None, U, VH, {Option.InnerBlocking: 64})
    assert (s.cpu() - torch.linalg.svdvals(Ad.cpu())).abs().max().item() < 1e-11
    assert (D(U) @ torch.diag(s.to(dev)) @ D(VH) - Ad).abs().max().item() < 1e-11


def _check_svd_grid(m, n, nb, dt, p, q, band):
    k = min(m, n)
    A = sl.Matrix(m, n, nb=nb, p=p, q=q, dtype=dt)
    A.insertLocalTiles()
    sl.generate_matrix(A, "rands", 7 + m)
    Ad = D(A).clone()
    U = sl.Matrix(m, k, nb=nb, p=p, q=q, dtype=dt)
    U.insertLocalTiles()
    VH = sl.Matrix(k, n, nb=nb, p=p, q=q, dtype=dt)
    VH.insertLocalTiles()
    s = sl.svd(A, None, U, VH, {Option.InnerBlocking: band})
    Ud, Vd = D(U), D(VH)
    sc = Ad.abs().max().item() * max(m, n)
    assert (s - torch.linalg.svdvals(Ad)).abs().max().item() < 1e-13 * sc
    assert (Ud @ torch.diag(s.to(dt)) @ Vd - Ad).abs().max().item() < 1e-13 * sc
    assert (Ud.mH @ Ud - torch.eye(k, dtype=dt)).abs().max().item() < 1e-12
    assert (Vd @ Vd.mH - torch.eye(k, dtype=dt)).abs().max().item() < 1e-12
    # values only, A untouched by the distributed path
    assert (D(A) - Ad).abs().max().item() == 0
    s2 = sl.svd_vals(A, None, {Option.InnerBlocking: band})
    assert (s2 - s).abs().max().item() < 1e-13 * sc


def _dist_svd_only(rank, size, p, q):
    _check_svd_grid(90, 60, 16, torch.float64, p, q, 8)
    _check_svd_grid(50, 77, 16, torch.float64, p, q, 16)
    _check_svd_grid(64, 64, 16, torch.complex128, p, q, 8)


@pytest.mark.parametrize("grid", [(2, 2), (4, 1), (1, 3)], ids=lambda g: f"{g[0]}x{g[1]}")
def test_svd_grid(grid):
    """ge2tb on the process grid (column QR + row LQ panels, no dense gather),
    band to rank 0 for tb2bd, bdsqr on each rank's own rows, grid
    back-transforms (V on the transposed grid)."""
    run_dist(_dist_svd_only, grid[0] * grid[1], *grid)


def test_svd_dist_path_one_rank(monkeypatch):
    monkeypatch.setenv("SLATE_AMD_SVD_DIST", "1")
    _check_svd_grid(70, 45, 16, torch.float64, 1, 1, 8)
    _check_svd_grid(33, 70, 16, torch.complex128, 1, 1, 16)


@pytest.mark.gpu
def test_svd_dist_path_gpu(monkeypatch):
    """The distributed SVD path on one GPU (HIP QR/GEMM/trmm kernels in
    ge2tb, device back-transforms)."""
    monkeypatch.setenv("SLATE_AMD_SVD_DIST", "1")
    dev = torch.device("cuda", 0)
    m, n, nb = 300, 200, 64
    A = sl.Matrix(m, n, nb=nb, device=dev)
    A.insertLocalTiles(device=0)
    sl.generate_matrix(A, "rands", 3)
    Ad = D(A).clone()
    U = sl.Matrix(m, n, nb=nb, device=dev)
    U.insertLocalTiles(device=0)
    VH = sl.Matrix(n, n, nb=nb, device=dev)
    VH.insertLocalTiles(device=0)
    s = sl.svd(A, None, U, VH, {Option.InnerBlocking: 32}).to(dev)
    assert ((D(U) @ torch.diag(s) @ D(VH) - Ad).abs().max() / (Ad.abs().max() * m)).item() < 1e-13


@pytest.mark.gpu
@pytest.mark.parametrize("dt,n,b", [(torch.float64, 300, 16), (torch.complex128, 200, 24), (torch.float64, 129, 64)])
def test_hb2st_gpu(dt, n, b, monkeypatch):
    """GPU bulge chasing (persistent ticket-ordered sweeps): tridiagonal
    eigenvalues = band eigenvalues, and Q2 T Q2^H reproduces the band."""
    monkeypatch.setenv("SLATE_AMD_HB2ST", "device")
    g = torch.Generator().manual_seed(3)
    X = torch.randn(n, n, generator=g, dtype=torch.float64).to(dt)
    if dt.is_complex:
        X = X + 1j * torch.randn(n, n, generator=g, dtype=torch.float64)
    H = X + X.mH
    i = torch.arange(n)
    H = torch.where((i[:, None] - i[None, :]).abs() <= b, H, torch.zeros_like(H))
    d, e, F = E.hb2st(H.clone(), b, device=torch.device("cuda"))
    w0 = torch.linalg.eigvalsh(H)
    T = torch.diag(d) + torch.diag(e, -1) + torch.diag(e, 1)
    assert (torch.linalg.eigvalsh(T) - w0).abs().max() / w0.abs().max() < 1e-13
    Z = ops.as_colmajor(torch.eye(n, dtype=dt).cuda()) if hasattr(ops, "as_colmajor") else torch.eye(n, dtype=dt).cuda()
    Z = Z.t().contiguous().t()
    E.unmtr_hb2st(F, Z)                               # Z = Q2 Phase
    Zc = Z.cpu()
    R = Zc @ T.to(dt) @ Zc.mH
    assert (R - H).abs().max() / H.abs().max() < 1e-12
    # the host pipeline gives the same tridiagonal spectrum
    monkeypatch.setenv("SLATE_AMD_HB2ST", "host")
    d2, e2, _ = E.hb2st(H.clone(), b, device=torch.device("cuda"))
    T2 = torch.diag(d2) + torch.diag(e2, -1) + torch.diag(e2, 1)
    assert (torch.linalg.eigvalsh(T2) - torch.linalg.eigvalsh(T)).abs().max() / w0.abs().max() < 1e-13


@pytest.mark.gpu
@pytest.mark.parametrize("leaf", [32, 128])
@pytest.mark.parametrize("n", [257, 3000])
def test_stedc_gpu_secular(n, leaf):
    """Merges on the GPU (secular roots / Gu-Eisenstat z / vectors by the
    stedc.hip kernels) vs an fp64 host reference."""
    torch.manual_seed(2)
    d, e = torch.randn(n, dtype=torch.float64), torch.randn(n - 1, dtype=torch.float64)
    T = torch.diag(d) + torch.diag(e, 1) + torch.diag(e, -1)
    wr = torch.linalg.eigvalsh(T)
    w, Z = sl.stedc(d, e, device="cuda", leaf=leaf)      # 128: two-wave leaf kernel
    Z = Z.cpu()
    tol = 1e-13 * n
    assert (w - wr).abs().max() < tol
    assert (T @ Z - Z * w).abs().max() < tol
    assert (Z.T @ Z - torch.eye(n, dtype=torch.float64)).abs().max() < tol
    d2 = torch.ones(n, dtype=torch.float64)
    d2[::3] = 2.0
    e2 = torch.full((n - 1,), 1e-9, dtype=torch.float64)
    T2 = torch.diag(d2) + torch.diag(e2, 1) + torch.diag(e2, -1)
    w, Z = sl.stedc(d2, e2, device="cuda", leaf=leaf)
    Z = Z.cpu()
    assert (T2 @ Z - Z * w).abs().max() < tol
    assert (Z.T @ Z - torch.eye(n, dtype=torch.float64)).abs().max() < tol


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["rand", "negative", "zero_e", "deflating", "clustered"])
def test_stedc_device_merge_one_sync_per_level(monkeypatch, case):
    """The level-batched device merges (sort, deflation, rotations and index
    sets on the GPU: stedc_level_prep) read the host ONCE per tree level and
    agree with the per-merge driver and an fp64 reference."""
    from slate_amd.models import stedc as SD
    n = 1500
    g = torch.Generator().manual_seed(7)
    d = torch.randn(n, dtype=torch.float64, generator=g)
    e = torch.randn(n - 1, dtype=torch.float64, generator=g)
    if case == "negative":
        e = -e.abs()
    elif case == "zero_e":
        e[::97] = 0.0
        e[500:700] = 0.0
    elif case == "deflating":
        d = torch.ones(n, dtype=torch.float64)
        d[::3] = 2.0
        e = torch.full((n - 1,), 1e-9, dtype=torch.float64)
    elif case == "clustered":
        d = torch.round(d * 4) / 4
        e = e * 1e-3
    T = torch.diag(d) + torch.diag(e, 1) + torch.diag(e, -1)
    wr = torch.linalg.eigvalsh(T)
    w, Z = sl.stedc(d, e, device="cuda", leaf=64)
    syncs, levels = SD.STEDC_STATS["host_syncs"], SD.STEDC_STATS["levels"]
    leaves, lv = SD._tree(n, 64)
    assert levels == len(lv) and syncs == levels, (SD.STEDC_STATS, len(lv))
    Z = Z.cpu()
    tol = 1e-13 * n
    assert (w - wr).abs().max() < tol * max(1.0, wr.abs().max())
    assert (T @ Z - Z * w).abs().max() < tol * max(1.0, wr.abs().max())
    assert (Z.T @ Z - torch.eye(n, dtype=torch.float64)).abs().max() < tol
    w2, _ = sl.stedc(d, e, device="cpu", leaf=64)          # the host per-merge path
    assert (w - w2).abs().max() < tol * max(1.0, wr.abs().max())


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float64, torch.complex128])
@pytest.mark.parametrize("n,b", [(300, 32), (517, 64), (200, 64), (1000, 64)])
def test_unmtr_hb2st_blocked_gpu(monkeypatch, dt, n, b):
    """One-launch blocked back-transform (blocks of b sweeps, sliding
    register window) == one launch per sweep."""
    g = torch.Generator().manual_seed(7)
    A = torch.randn(n, n, dtype=dt, generator=g)
    A = A + A.mH
    i = torch.arange(n)
    A = torch.where((i[:, None] - i[None, :]).abs() <= b, A, torch.zeros_like(A))
    d, e, F = E.hb2st(E._cm(A.clone()), b)
    Z0 = torch.randn(n, 77, dtype=dt, generator=g)
    Za = E._cm(Z0.cuda())
    Zb = E._cm(Z0.cuda())
    monkeypatch.setenv("SLATE_AMD_UNMTR_BLOCKED", "0")
    E.unmtr_hb2st(F, Za)
    monkeypatch.setenv("SLATE_AMD_UNMTR_BLOCKED", "1")
    monkeypatch.setenv("SLATE_AMD_UNMTR_MFMA", "0")
    E.unmtr_hb2st(F, Zb)
    assert (Za - Zb).abs().max().item() < 1e-12 * n
    # block reflectors on MFMA (real, b = 64)
    Zc = E._cm(Z0.cuda())
    monkeypatch.setenv("SLATE_AMD_UNMTR_MFMA", "1")
    E.unmtr_hb2st(F, Zc)
    assert (Za - Zc).abs().max().item() < 1e-12 * n


@pytest.mark.parametrize("dt", [torch.float64, torch.complex128])
@pytest.mark.parametrize("n,b", [(150, 8), (97, 3), (64, 1), (40, 16)])
def test_tb2bd_pipelined_equals_sequential(dt, n, b, monkeypatch):
    """The multi-threaded pipelined chase (sweep j waits for sweep j-1's
    progress counter) is bitwise the sequential one (src/tb2bd.cc task
    graph): same bidiagonal, same reflectors in the same slots."""
    g = torch.Generator().manual_seed(n + b)
    A = torch.randn(n, n, dtype=dt, generator=g)
    i = torch.arange(n)
    dlt = i[None, :] - i[:, None]
    A = torch.where((dlt >= 0) & (dlt <= b), A, torch.zeros_like(A))
    out = []
    for th in ("1", "6"):
        monkeypatch.setenv("SLATE_AMD_TB2BD_THREADS", th)
        d, e, F = S.tb2bd(A.clone(), b)
        out.append((d, e, F))
    (d1, e1, F1), (d2, e2, F2) = out
    assert torch.equal(d1, d2) and torch.equal(e1, e2)
    for a, c in ((F1.U, F2.U), (F1.V, F2.V)):
        assert torch.equal(a.V, c.V) and torch.equal(a.tau, c.tau)
    # and it is a bidiagonalisation: singular values preserved
    s_ref = torch.linalg.svdvals(A)
    Bd = torch.diag(d1) + torch.diag(e1, 1)
    assert torch.allclose(torch.linalg.svdvals(Bd), s_ref, atol=1e-12 * s_ref[0].item())


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float64, torch.complex128])
@pytest.mark.parametrize("n,b", [(300, 8), (257, 64), (100, 1), (130, 128)])
def test_tb2bd_gpu_equals_host(dt, n, b, monkeypatch):
    """GPU bidiagonal chase (tight windows, persistent workgroups) against
    the host pipeline: same bidiagonal and reflectors to rounding."""
    g = torch.Generator().manual_seed(n * b)
    A = torch.randn(n, n, dtype=dt, generator=g)
    i = torch.arange(n)
    dlt = i[None, :] - i[:, None]
    A = torch.where((dlt >= 0) & (dlt <= b), A, torch.zeros_like(A))
    d1, e1, F1 = S.tb2bd(A.clone(), b)
    d2, e2, F2 = S.tb2bd(A.clone().cuda(), b)
    sc = A.abs().max().item() * n
    # different summation orders (host: serial, device: quad-lane partial sums)
    assert (d1 - d2).abs().max().item() < 1e-12 * sc
    assert (e1 - e2).abs().max().item() < 1e-12 * sc
    for a, c in ((F1.U, F2.U), (F1.V, F2.V)):
        assert a.count == c.count
        assert torch.equal(a.row, c.row.cpu()) and torch.equal(a.length, c.length.cpu())
    # the device reflectors reproduce the band (reflectors of near-zero
    # columns are only defined to rounding, so compare their action):
    # A = Q_U diag(pu) B diag(pv)^H Q_V^H with B the real bidiagonal
    QU = E.unmtr_hb2st(F2.U, torch.eye(n, dtype=dt, device="cuda").t())
    QV = E.unmtr_hb2st(F2.V, torch.eye(n, dtype=dt, device="cuda").t())
    Bd = (torch.diag(d2) + torch.diag(e2, 1)).to(dt)
    R = QU.cpu() @ torch.diag(F2.pu) @ Bd @ torch.diag(F2.pv).mH @ QV.cpu().mH - A
    assert R.abs().max().item() < 1e-13 * sc


@pytest.mark.gpu
def test_svd_gpu_complex():
    dev = torch.device("cuda")
    m, n = 260, 200
    A = sl.Matrix(m, n, nb=64, dtype=torch.complex128, device=dev)
    A.insertLocalTiles(device=0)
    sl.generate_matrix(A, "rands", 11)
    Ad = D(A).clone()
    U = sl.Matrix(m, n, nb=64, dtype=torch.complex128, device=dev)
    U.insertLocalTiles(device=0)
    VH = sl.Matrix(n, n, nb=64, dtype=torch.complex128, device=dev)
    VH.insertLocalTiles(device=0)
    s = sl.svd(A, None, U, VH, {Option.InnerBlocking: 32})
    assert (s.cpu() - torch.linalg.svdvals(Ad.cpu())).abs().max().item() < 1e-11
    assert (D(U) @ torch.diag(s.to(dev).to(torch.complex128)) @ D(VH) - Ad).abs().max().item() < 1e-11


def _stedc_rows_dist(rank, size):
    """Distributed D&C (models/stedc.py): each rank holds only its block of
    rows of the eigenvector matrix -- never n x n -- and the gathered result
    is an orthonormal eigenbasis of the tridiagonal."""
    import numpy as np
    from slate_amd.models.stedc import stedc_rows
    from slate_amd.parallel.comm import world
    comm = world()
    for n, seed in ((301, 0), (129, 1), (64, 2)):
        rng = np.random.default_rng(seed)
        d, e = rng.standard_normal(n), rng.standard_normal(n - 1)
        if seed == 1:                       # clustered spectrum: Givens deflation chains
            d = np.round(d, 1)
            e[::3] = 1e-12
        w, Q, r0, r1, mb = stedc_rows(d, e, comm, "cpu", leaf=16)
        assert Q.shape == (r1 - r0, n) and r1 - r0 <= -(-n // size)
        rows = comm.allgather(torch.nn.functional.pad(Q, (0, 0, 0, mb - Q.shape[0])).contiguous())
        Z = rows.reshape(size * mb, n)[:n]
        T = torch.diag(torch.from_numpy(d)) + torch.diag(torch.from_numpy(e), 1) + torch.diag(torch.from_numpy(e), -1)
        ref = torch.linalg.eigvalsh(T)
        assert float((w - ref).abs().max()) < 1e-12 * n
        assert float((T @ Z - Z * w).abs().max()) < 1e-12 * n
        assert float((Z.T @ Z - torch.eye(n, dtype=torch.float64)).abs().max()) < 1e-12 * n


@pytest.mark.parametrize("size", [2, 3, 4])
def test_stedc_rows_distributed(size):
    run_dist(_stedc_rows_dist, size)


def test_stedc_rows_one_rank():
    import numpy as np
    from slate_amd.models.stedc import stedc_rows
    n = 257
    rng = np.random.default_rng(5)
    d, e = rng.standard_normal(n), rng.standard_normal(n - 1)
    w, Q, r0, r1, _ = stedc_rows(d, e, None, "cpu", leaf=32)
    T = torch.diag(torch.from_numpy(d)) + torch.diag(torch.from_numpy(e), 1) + torch.diag(torch.from_numpy(e), -1)
    assert (r0, r1) == (0, n)
    assert float((T @ Q - Q * w).abs().max()) < 1e-12 * n


def test_stedc_leaf_nonconvergence_raises(monkeypatch):
    """a leaf QL that hits its iteration cap must not return
    wrong eigenpairs silently -- stedc raises with info = #failed leaves."""
    import numpy as np
    from slate_amd.core.exceptions import NumericalError
    from slate_amd.models.stedc import stedc_rows
    monkeypatch.setenv("SLATE_AMD_STEQR_MAXIT", "0")
    rng = np.random.default_rng(6)
    n = 100
    d, e = rng.standard_normal(n), rng.standard_normal(n - 1)
    with pytest.raises(NumericalError) as ei:
        stedc_rows(d, e, None, "cpu", leaf=32)
    assert ei.value.info >= 1


@pytest.mark.gpu
def test_stedc_leaf_nonconvergence_raises_gpu(monkeypatch):
    import numpy as np
    from slate_amd.core.exceptions import NumericalError
    from slate_amd.models.stedc import stedc_rows
    monkeypatch.setenv("SLATE_AMD_STEQR_MAXIT", "0")
    rng = np.random.default_rng(6)
    n = 300
    d, e = rng.standard_normal(n), rng.standard_normal(n - 1)
    with pytest.raises(NumericalError):
        stedc_rows(d, e, None, "cuda")


@pytest.mark.gpu
@pytest.mark.parametrize("early,lag,reuse", [("1", "3", "1"), ("1", "3", "0"), ("0", "3", "0"), ("0", "4", "0")])
def test_hb2st_gpu_matches_host_chase(early, lag, reuse, monkeypatch):
    """The pipelined GPU chase equals the sequential host chase up to the
    summation order inside a task: a dependency rule (early publication of
    a task's annihilated entries, or a lag of whole tasks) that let
    overlapping tasks of two sweeps run out of order would change the
    tridiagonal entries, not only round them (n = 2000 with b = 64: 31 tasks
    in the first sweep, up to ~24 sweeps in flight)."""
    monkeypatch.setenv("SLATE_AMD_HB2ST_EARLY", early)
    monkeypatch.setenv("SLATE_AMD_HB2ST_LAG", lag)
    monkeypatch.setenv("SLATE_AMD_HB2ST_REUSE", reuse)      # sweep-resident window (early mode only)
    n, b = 2000, 64
    g = torch.Generator().manual_seed(11)
    X = torch.randn(n, n, generator=g, dtype=torch.float64)
    H = X + X.T
    i = torch.arange(n)
    H = torch.where((i[:, None] - i[None, :]).abs() <= b, H, torch.zeros_like(H))
    monkeypatch.setenv("SLATE_AMD_HB2ST", "device")
    d, e, _ = E.hb2st(H.clone(), b, device=torch.device("cuda"))
    monkeypatch.setenv("SLATE_AMD_HB2ST", "host")
    d2, e2, _ = E.hb2st(H.clone(), b, device=torch.device("cuda"))
    scale = H.abs().max().item()
    assert (d.cpu() - d2.cpu()).abs().max().item() / scale < 1e-11
    assert (e.cpu().abs() - e2.cpu().abs()).abs().max().item() / scale < 1e-11


@pytest.mark.parametrize("group", ["1", "3", "4", "8"])
@pytest.mark.parametrize("dt", [torch.float64, torch.complex128])
def test_unmtr_he2hb_grouped_panels(group, dt, monkeypatch):
    """Stage-1 back-transform with consecutive panels merged into one block
    reflector (forward larft merge) equals the panel-by-panel application."""
    from slate_amd.models.qr import _apply_qh
    monkeypatch.setenv("SLATE_AMD_UNMTR_HE2HB_GROUP", group)
    n, nb = 260, 16
    g = torch.Generator().manual_seed(5)
    X = torch.randn(n, n, generator=g, dtype=torch.float64).to(dt)
    if dt.is_complex:
        X = X + 1j * torch.randn(n, n, generator=g, dtype=torch.float64)
    H = (X + X.mH).t().contiguous().t()
    F = E.he2hb(H.clone().t().contiguous().t(), nb)
    Z0 = torch.randn(n, 9, generator=g, dtype=torch.float64).to(dt).t().contiguous().t()
    Za = Z0.clone().t().contiguous().t()
    for (r0, V, T) in reversed(F.panels):
        _apply_qh(V, T, Za[r0:, :], conj=False)
    Zb = E.unmtr_he2hb(F, Z0.clone().t().contiguous().t())
    assert (Za - Zb).abs().max().item() < 1e-12
