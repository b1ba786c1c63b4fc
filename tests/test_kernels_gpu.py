"""gfx950 kernel numerics vs fp64 PyTorch references (unit tests
of every device kernel against a host reference, unit_test/test_geadd.cc &c)."""
import pytest
import torch

from slate_amd import ops, _native

pytestmark = pytest.mark.gpu
DT = [torch.float64, torch.float32, torch.complex128, torch.complex64]
TOL = {torch.float64: 1e-12, torch.float32: 2e-5, torch.complex128: 1e-12, torch.complex64: 2e-5}


def cm(m, n, dt, seed=0, dev="cuda"):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(n, m, dtype=dt, generator=g).t()
    return _cm(x, dev)


def _cm(x, dev):
    y = torch.empty((x.shape[1], x.shape[0]), dtype=x.dtype, device=dev).t()
    y.copy_(x)
    return y


def ref(x):
    return x.to(torch.complex128 if x.dtype.is_complex else torch.float64)


def opx(x, t):
    return {'N': x, 'T': x.mT, 'C': x.mH}[t]


def test_native_loaded():
    assert _native._hip is not None
    assert _native._hip.arch == "gfx950"


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("ta,tb", [("N", "N"), ("N", "T"), ("T", "N"), ("C", "C"), ("N", "C")])
def test_gemm(dt, ta, tb):
    if not dt.is_complex and "C" in (ta + tb):
        pytest.skip("conj on real")
    m, n, k = 197, 131, 77
    A = cm(k, m, dt, 1) if ta != 'N' else cm(m, k, dt, 1)
    B = cm(n, k, dt, 2) if tb != 'N' else cm(k, n, dt, 2)
    C = cm(m, n, dt, 3)
    R = 0.7 * ref(opx(A, ta)) @ ref(opx(B, tb)) - 0.3 * ref(C)
    ops.gemm(0.7, A, B, -0.3, C, ta, tb)
    assert (ref(C) - R).abs().max() / R.abs().max() < TOL[dt]


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("tt", ["TN", "NN", "NT"])
@pytest.mark.parametrize("mnk", [(200, 96, 20000 + 37), (64, 4100, 6000 + 13), (3000, 64, 4096)])
def test_gemm_splitk(dt, tt, mnk):
    # few output tiles + long k -> split-K path (+ ragged last chunk); the
    # wide 64-row / 64-column shapes take the fp64 split for <= 512 64 x 64 tiles
    ta, tb = tt[0], tt[1]
    if dt.is_complex:
        ta = 'C' if ta == 'T' else ta
    m, n, k = mnk
    A = cm(k, m, dt, 1) if ta != 'N' else cm(m, k, dt, 1)
    B = cm(n, k, dt, 2) if tb != 'N' else cm(k, n, dt, 2)
    C = cm(m, n, dt, 3)
    R = 0.5 * ref(opx(A, ta)) @ ref(opx(B, tb)) + 2.0 * ref(C)
    ops.gemm(0.5, A, B, 2.0, C, ta, tb)
    assert (ref(C) - R).abs().max() / R.abs().max() < 4 * TOL[dt]


def test_gemm_large_k512():
    m = n = 2048
    A, B, C = cm(m, 512, torch.float64, 4), cm(n, 512, torch.float64, 5), cm(m, n, torch.float64, 6)
    R = ref(C) - A @ B.mT
    ops.gemm(-1.0, A, B, 1.0, C, 'N', 'T')
    assert (C - R).abs().max() < 1e-11


def test_gemm_trimask_blockcyclic():
    # lower mask in global coords of a 2x? block-cyclic local buffer (pr=1 of p=2, nb=64)
    nb, p, pr = 64, 2, 1
    m = n = 256
    A, B, C = cm(m, 32, torch.float64, 7), cm(n, 32, torch.float64, 8), cm(m, n, torch.float64, 9)
    C0 = C.clone()
    ops.gemm(1.0, A, B, 1.0, C, 'N', 'T', mask=(1, nb, p, pr, p, pr, 0, 0, 0))
    full = C0 + A @ B.mT
    gr = torch.tensor([((i // nb) * p + pr) * nb + i % nb for i in range(m)], device="cuda")
    keep = gr[:, None] >= gr[None, :]
    exp = torch.where(keep, full, C0)
    assert (C - exp).abs().max() < 1e-12


@pytest.mark.parametrize("m,n,roff,coff,doff", [
    (256, 256, 0, 0, 0), (1000, 700, 0, 0, 0), (700, 1000, 0, 0, 0), (900, 900, 0, 128, 0),
    (900, 900, 64, 64, -5), (6400, 6400, 0, 0, 0), (6500, 6300, 0, 0, 0), (6400, 6400, 0, 256, 0)])
def test_gemm_trimask_compact(m, n, roff, coff, doff):
    # one-rank lower mask: compact lower-triangle launch (remap = 2) for both
    # fp64 tile variants (64 x 64 below 2048 128-tiles, 128 x 128 above)
    A, B, C = cm(m, 32, torch.float64, 7), cm(n, 32, torch.float64, 8), cm(m, n, torch.float64, 9)
    C0 = C.clone()
    ops.gemm(1.0, A, B, 1.0, C, 'N', 'T', mask=(1, 1 << 40, 1, 0, 1, 0, roff, coff, doff))
    full = C0 + A @ B.mT
    r = torch.arange(m, device="cuda")[:, None] + roff
    c = torch.arange(n, device="cuda")[None, :] + coff
    exp = torch.where(r + doff >= c, full, C0)
    assert (C - exp).abs().max() < 1e-12


@pytest.mark.parametrize("p,pr,q,pc,roff,coff", [
    (2, 1, 4, 2, 0, 0), (2, 0, 4, 3, 256, 512), (1, 0, 2, 1, 0, 0), (2, 1, 1, 0, 0, 0), (2, 0, 2, 0, 512, 256)])
def test_gemm_trimask_compact_blockcyclic(p, pr, q, pc, roff, coff):
    # block-cyclic lower mask, 128 x 128 tiles: the compact launch where no
    # tile above the tile diagonal is live (p <= q), full grid otherwise
    nb, m, n = 512, 6400, 6144
    A, B, C = cm(m, 32, torch.float64, 7), cm(n, 32, torch.float64, 8), cm(m, n, torch.float64, 9)
    C0 = C.clone()
    ops.gemm(1.0, A, B, 1.0, C, 'N', 'T', mask=(1, nb, p, pr, q, pc, roff, coff, 0))
    full = C0 + A @ B.mT
    lr = torch.arange(m, device="cuda") + roff
    lc = torch.arange(n, device="cuda") + coff
    gr = ((lr // nb) * p + pr) * nb + lr % nb
    gc = ((lc // nb) * q + pc) * nb + lc % nb
    exp = torch.where(gr[:, None] >= gc[None, :], full, C0)
    assert (C - exp).abs().max() < 1e-12


@pytest.mark.parametrize("p,pr,q,pc,m,n", [
    (1, 0, 2, 0, 32256, 15872), (1, 0, 2, 1, 20000, 9000), (2, 0, 1, 0, 15872, 31744), (4, 1, 2, 1, 3000, 2500),
    (1, 0, 4, 2, 1500, 700)])
def test_gemm_stair_exact_grid(p, pr, q, pc, m, n):
    # the exact staircase launch (remap 4: host prefix sums per row group,
    # binary searches per block) on tall / wide / ragged local blocks, both
    # tile sizes; every kept element updated once, every skipped one intact
    nb = 512
    A, B, C = cm(m, 16, torch.float64, 7), cm(n, 16, torch.float64, 8), cm(m, n, torch.float64, 9)
    C0 = C.clone()
    ops.gemm(1.0, A, B, 1.0, C, 'N', 'T', mask=(1, nb, p, pr, q, pc, 0, 0, 0))
    full = C0 + A @ B.mT
    lr = torch.arange(m, device="cuda")
    lc = torch.arange(n, device="cuda")
    gr = ((lr // nb) * p + pr) * nb + lr % nb
    gc = ((lc // nb) * q + pc) * nb + lc % nb
    exp = torch.where(gr[:, None] >= gc[None, :], full, C0)
    assert (C - exp).abs().max() < 1e-12


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("uplo", ["L", "U"])
def test_potrf_tile(dt, uplo):
    n = 300
    X = ref(cm(n, n, dt, 11))
    S = X @ X.mH + n * torch.eye(n, dtype=X.dtype, device=X.device)
    A = _cm(S.to(dt), "cuda")
    info = ops.potrf(uplo, A)
    assert int(info.item()) == 0
    L = torch.tril(ref(A)) if uplo == 'L' else torch.triu(ref(A))
    R = L @ L.mH if uplo == 'L' else L.mH @ L
    assert (R - S).abs().max() / S.abs().max() < 10 * TOL[dt]


def test_potrf_tile_info():
    n = 64
    S = torch.eye(n, dtype=torch.float64, device="cuda")
    S[40, 40] = -1.0
    A = _cm(S, "cuda")
    assert int(ops.potrf('L', A).item()) == 41


@pytest.mark.parametrize("n", [1, 17, 32, 33, 100, 511, 512, 513, 1100])
def test_potrf_tile_fp64_fast(n):
    # one-CU LDS kernel (n <= 512) and its 512-blocked composition (n > 512);
    # ragged 16/32-column edges, lda > n
    X = ref(cm(n, n, torch.float64, 31))
    S = X @ X.mT + n * torch.eye(n, dtype=torch.float64, device="cuda")
    Abig = _cm(torch.zeros(n + 7, n, dtype=torch.float64, device="cuda"), "cuda")
    Abig[:n].copy_(S)
    A = Abig[:n]
    info = ops.potrf('L', A)
    assert int(info.item()) == 0
    L = torch.tril(A)
    assert (L @ L.mT - S).abs().max() / S.abs().max() < 1e-14
    assert (torch.triu(A, 1) == torch.triu(S, 1)).all()          # upper triangle untouched


@pytest.mark.parametrize("bad", [0, 15, 16, 40, 300])
def test_potrf_tile_fp64_fast_info(bad):
    n = 320
    S = 4.0 * torch.eye(n, dtype=torch.float64, device="cuda")
    S[bad, bad] = -1.0
    A = _cm(S, "cuda")
    assert int(ops.potrf('L', A).item()) == bad + 1


@pytest.mark.parametrize("m,n", [(1, 1), (64, 32), (65, 33), (1000, 512), (4097, 100), (300, 1000)])
@pytest.mark.parametrize("diag", ["N", "U"])
@pytest.mark.parametrize("ks", ["1", "2", "4"])
def test_trsm_rlt_fp64_fast(m, n, diag, ks, monkeypatch):
    # X L^T = alpha B: the Cholesky panel solve (tri_inv32 + trsm_rlt kernels;
    # SLATE_AMD_TRSM_KS: the K-split variants, 32- and 16-row blocks)
    monkeypatch.setenv("SLATE_AMD_TRSM_KS", ks)
    T = torch.tril(ref(cm(n, n, torch.float64, 41))) / n + 2 * torch.eye(n, dtype=torch.float64, device="cuda")
    Tu = T.clone()
    if diag == 'U':
        Tu.diagonal().fill_(1)
    A = _cm(T, "cuda")
    B = cm(m, n, torch.float64, 42)
    B0 = B.clone()
    ops.trsm('R', 'L', 'T', diag, -1.5, A, B)
    assert ((B @ Tu.mT) + 1.5 * B0).abs().max() / B0.abs().max() < 1e-12


@pytest.mark.parametrize("dt", [torch.float64, torch.complex128, torch.float32])
@pytest.mark.parametrize("side", ["L", "R"])
@pytest.mark.parametrize("uplo", ["L", "U"])
@pytest.mark.parametrize("trans", ["N", "T", "C"])
@pytest.mark.parametrize("diag", ["N", "U"])
def test_trsm_trmm(dt, side, uplo, trans, diag):
    m, n = 150, 97
    k = m if side == 'L' else n
    T = ref(cm(k, k, dt, 21)) / k + 2 * torch.eye(k, device="cuda")
    T = torch.tril(T) if uplo == 'L' else torch.triu(T)
    Tu = T.clone()
    if diag == 'U':
        Tu.diagonal().fill_(1)
    A = _cm(T.to(dt), "cuda")
    B = cm(m, n, dt, 22)
    B0 = ref(B).clone()
    ops.trsm(side, uplo, trans, diag, 2.0, A, B)
    oT = opx(Tu, trans)
    X = ref(B)
    R = oT @ X if side == 'L' else X @ oT
    assert (R - 2 * B0).abs().max() / B0.abs().max() < 100 * TOL[dt]
    B2 = _cm(B0.to(dt), "cuda")
    ops.trmm(side, uplo, trans, diag, 1.5, A, B2)
    R2 = 1.5 * (oT @ B0 if side == 'L' else B0 @ oT)
    assert (ref(B2) - R2).abs().max() / R2.abs().max() < 100 * TOL[dt]


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("m,n", [(1000, 96), (300, 300), (64, 100), (2000, 33)])
def test_getrf_panel(dt, m, n):
    A0 = ref(cm(m, n, dt, 31)).clone()
    A = _cm(A0.to(dt), "cuda")
    k = min(m, n)
    ipiv = torch.zeros(k, dtype=torch.int64, device="cuda")
    info = ops.getrf(A, ipiv)
    assert int(info.item()) == 0
    LU = ref(A)
    L = torch.tril(LU[:, :k], -1) + torch.eye(m, k, dtype=LU.dtype, device="cuda")
    U = torch.triu(LU[:k, :])
    P = A0.clone()
    for i, p in enumerate(ipiv.tolist()):
        if p != i:
            P[[i, p]] = P[[p, i]]
    assert (L @ U - P).abs().max() / A0.abs().max() < 100 * TOL[dt]
    # partial pivoting (cabs1 as LAPACK izamax): |re(l)| + |im(l)| <= 1
    bound = 2.0 if L.is_complex() else 1.0   # cabs1 pivoting bounds |l| by sqrt(2) -> cabs1(l) <= 2
    assert (L.real.abs() + (L.imag.abs() if L.is_complex() else 0)).max() <= bound + 1e-6


@pytest.mark.parametrize("m,n", [(2048, 32), (5000, 64), (20000, 100), (32768, 512)])
def test_getrf_panel_persistent_fp64(m, n):
    # tall fp64 panels take the persistent base case (co-resident workgroups,
    # sc1 hand-offs); pivots must equal LAPACK's partial pivoting exactly
    A0 = cm(m, n, torch.float64, 33)
    A = A0.clone()
    ipiv = torch.zeros(n, dtype=torch.int64, device="cuda")
    info = ops.getrf(A, ipiv)
    assert int(info.item()) == 0
    LU_ref, piv_ref = torch.linalg.lu_factor(A0.cpu())
    assert torch.equal(ipiv.cpu(), piv_ref[:n].to(torch.int64) - 1)
    assert (A.cpu() - LU_ref).abs().max() / A0.abs().max() < 1e-12


@pytest.mark.parametrize("m,n", [(65536, 64), (40000, 96)])
def test_getrf_panel_persistent_two_rows_per_thread(m, n):
    # 32768 < m <= 65536: each persistent thread holds two rows
    A0 = cm(m, n, torch.float64, 36)
    A = A0.clone()
    ipiv = torch.zeros(n, dtype=torch.int64, device="cuda")
    before = _native.hip().lu_persist_fallbacks()
    info = ops.getrf(A, ipiv)
    assert int(info.item()) == 0
    assert _native.hip().lu_persist_fallbacks() == before          # took the persistent path
    LU_ref, piv_ref = torch.linalg.lu_factor(A0.cpu())
    assert torch.equal(ipiv.cpu(), piv_ref[:n].to(torch.int64) - 1)
    assert (A.cpu() - LU_ref).abs().max() / A0.abs().max() < 1e-12


@pytest.mark.parametrize("m,n", [(5000, 64), (32768, 96)])
def test_getrf_panel_persistent_abort_falls_back(m, n):
    # a launch whose workgroups are not co-resident aborts by consensus and
    # the CAS winner refactors the block alone: same pivots, same factors,
    # counted in lu_persist_fallbacks (forced here through the test knob)
    H = _native.hip()
    A0 = cm(m, n, torch.float64, 37)
    A = A0.clone()
    ipiv = torch.zeros(n, dtype=torch.int64, device="cuda")
    before = H.lu_persist_fallbacks(1)
    try:
        info = ops.getrf(A, ipiv)
        torch.cuda.synchronize()
    finally:
        after = H.lu_persist_fallbacks(0)
    assert after > before
    assert int(info.item()) == 0
    LU_ref, piv_ref = torch.linalg.lu_factor(A0.cpu())
    assert torch.equal(ipiv.cpu(), piv_ref[:n].to(torch.int64) - 1)
    assert (A.cpu() - LU_ref).abs().max() / A0.abs().max() < 1e-12


def test_getrf_panel_persistent_abort_reports_singular():
    H = _native.hip()
    m, n = 3000, 40
    A0 = cm(m, n, torch.float64, 38)
    A0[:, 7] = 0.0
    A = A0.clone()
    ipiv = torch.zeros(n, dtype=torch.int64, device="cuda")
    H.lu_persist_fallbacks(1)
    try:
        info = ops.getrf(A, ipiv)
        torch.cuda.synchronize()
    finally:
        H.lu_persist_fallbacks(0)
    assert int(info.item()) == 8


@pytest.mark.parametrize("m,n", [(16, 1), (32, 32), (45, 7), (64, 64), (64, 1000), (100, 50), (256, 300), (512, 4000), (1000, 70)])
@pytest.mark.parametrize("unit", [False, True])
def test_trsm_lln_fp64_fast(m, n, unit):
    # L X = alpha B (lower, no-trans): one-launch blocked-inverse MFMA kernel
    g = torch.Generator().manual_seed(m + n)
    Lf = torch.randn(m + 5, m, dtype=torch.float64, generator=g)
    Lf[:m] = torch.tril(Lf[:m]) + 2 * m ** 0.5 * torch.eye(m, dtype=torch.float64)
    L = Lf.t().contiguous().t().cuda()[:m]                # lda > m
    B0 = torch.randn(m, n, dtype=torch.float64, generator=g)
    B = B0.t().contiguous().t().cuda()
    ops.trsm('L', 'L', 'N', 'U' if unit else 'N', 0.5, L, B)
    Lr = torch.tril(Lf[:m], -1) + torch.eye(m, dtype=torch.float64) if unit else torch.tril(Lf[:m])
    X = torch.linalg.solve_triangular(Lr, 0.5 * B0, upper=False, unitriangular=unit)
    assert (B.cpu() - X).abs().max() / X.abs().max() < 1e-12


@pytest.mark.parametrize("m,n", [(20000, 64), (32768, 256)])
def test_getrf_panel_persistent_under_load(m, n):
    # granule hand-offs while a GEMM streams on another stream (uneven
    # progress across the persistent workgroups): results must not change
    X = cm(6144, 6144, torch.float64, 5)
    side = torch.cuda.Stream()
    A0 = cm(m, n, torch.float64, 35)
    A = A0.clone()
    ipiv = torch.zeros(n, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        for _ in range(3):
            X = (X @ X) * (1.0 / 6144)
    info = ops.getrf(A, ipiv)
    torch.cuda.synchronize()
    assert int(info.item()) == 0
    LU_ref, piv_ref = torch.linalg.lu_factor(A0.cpu())
    assert torch.equal(ipiv.cpu(), piv_ref[:n].to(torch.int64) - 1)
    assert (A.cpu() - LU_ref).abs().max() / A0.abs().max() < 1e-12


@pytest.mark.parametrize("ns,m,incx", [(1, 5, 1), (32, 40, 1), (512, 2000, 1), (700, 3000, 1), (300, 900, -1),
                                       (1100, 5000, -1)])
def test_laswp_random_sequences(ns, m, incx):
    # parallel fold of the swap sequence (chains of repeated targets) vs sequential
    g = torch.Generator().manual_seed(ns + m)
    span = torch.randint(0, 4, (ns,), generator=g)
    far = torch.randint(0, m, (ns,), generator=g)
    ipiv = torch.tensor([min(m - 1, k + (int(far[k]) if span[k] == 3 else int(span[k]))) for k in range(ns)],
                        dtype=torch.int64)
    ipiv = torch.maximum(ipiv, torch.arange(ns))
    A0 = cm(m, 7, torch.float64, 43)
    A = A0.clone()
    ops.laswp(A, ipiv.cuda(), 0, ns, incx=incx)
    R = A0.clone()
    order = range(ns) if incx > 0 else reversed(range(ns))
    for i in order:
        p = int(ipiv[i])
        R[[i, p]] = R[[p, i]]
    assert torch.equal(A, R)


def test_laswp_matches_sequential():
    m, n = 600, 70
    A0 = cm(m, n, torch.float64, 41)
    ipiv = torch.tensor([(i * 37 + 5) % m for i in range(200)], dtype=torch.int64)
    ipiv = torch.maximum(ipiv, torch.arange(200))
    A = A0.clone()
    ops.laswp(A, ipiv.cuda(), 0, 200)
    R = A0.clone()
    for i, p in enumerate(ipiv.tolist()):
        R[[i, p]] = R[[p, i]]
    assert torch.equal(A, R)


@pytest.mark.parametrize("dt", DT)
def test_aux_kernels(dt):
    m, n = 130, 70
    A, B = cm(m, n, dt, 51), cm(m, n, dt, 52)
    B0 = B.clone()
    ops.geadd(2.0, A, 0.5, B)
    assert (B - (2 * A + 0.5 * B0)).abs().max() < 1e-5
    ops.gescale(3.0, B, uplo='L')
    ops.geset(1.5, -2.0, A, uplo='U')
    assert (torch.triu(A, 1) - torch.triu(torch.full_like(A, 1.5), 1)).abs().max() == 0
    assert (torch.diagonal(A) + 2).abs().max() == 0
    C = ops.colmajor_empty(n, m, dt, "cuda")
    ops.gecopy(B0, C, trans='C' if dt.is_complex else 'T')
    assert torch.equal(C, B0.mH if dt.is_complex else B0.mT)


@pytest.mark.parametrize("dt", DT)
def test_norm_local(dt):
    m, n = 257, 129
    A = cm(m, n, dt, 61)
    a = ref(A).abs()
    c, _ = ops.genorm_local('M', A)
    assert abs(c.max().item() - a.max().item()) < 1e-5
    c, _ = ops.genorm_local('1', A)
    assert (c - a.sum(0).to(c.dtype)).abs().max() < 1e-4
    _, r = ops.genorm_local('I', A)
    assert (r - a.sum(1).to(r.dtype)).abs().max() < 1e-4
    c, _ = ops.genorm_local('F', A)
    fro = (c[:, 0] ** 2 * c[:, 1]).sum().sqrt()
    assert abs(fro.item() - torch.linalg.norm(ref(A)).item()) < 1e-4 * fro.item()


@pytest.mark.parametrize("dt", DT)
def test_matgen_device_equals_host(dt):
    m, n, nb = 100, 90, 32
    for kind in (11, 21, 12):
        H = torch.zeros((n, m), dtype=dt).t()
        D = torch.zeros((n, m), dtype=dt, device="cuda").t()
        ops.matgen(kind, 1234, H, m, n, nb, 1, 0, nb, 1, 0)
        ops.matgen(kind, 1234, D, m, n, nb, 1, 0, nb, 1, 0)
        assert (D.cpu() - H).abs().max() < 1e-6


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("depth", [1, 2, 4])
def test_butterfly_gpu(dt, depth):
    """One-pass RBT kernel (all levels in registers) vs the explicit dense
    butterfly product, rows and column index, W and W^T."""
    from slate_amd.models.mixed import _butterfly_diag
    n, m = 256, 40
    dg = _butterfly_diag(n, depth, 5)
    W = torch.eye(n, dtype=torch.float64)
    for lvl in range(depth):
        size, Wl = n >> lvl, torch.zeros(n, n, dtype=torch.float64)
        h = size // 2
        i = torch.arange(h)
        for o in range(0, n, size):
            r0, r1 = dg[lvl, o + i], dg[lvl, o + h + i]
            Wl[o + i, o + i], Wl[o + i, o + h + i] = r0, r1
            Wl[o + h + i, o + i], Wl[o + h + i, o + h + i] = r0, -r1
        W = (Wl / 2 ** 0.5) @ W
    rdt = torch.float32 if dt in (torch.float32, torch.complex64) else torch.float64
    X, Y = cm(n, m, dt, 1), cm(m, n, dt, 2)
    for trans in (False, True):
        opW = (W.mT if trans else W).to(ref(X).dtype).cuda()
        got = ops.butterfly(X.clone(), dg.to(rdt).cuda(), depth, trans, 'L')
        assert (ref(got) - opW @ ref(X)).abs().max().item() < TOL[dt] * 10
        got = ops.butterfly(Y.clone(), dg.to(rdt).cuda(), depth, trans, 'R')
        assert (ref(got) - ref(Y) @ opW.mT).abs().max().item() < TOL[dt] * 10


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float64, torch.complex128])
def test_gelqf_panel_device_matches_host(dt):
    """ops.gelqf on the device (QR of A^H) gives the host LQ: same L and
    tau (LAPACK layout)."""
    from slate_amd import ops
    g = torch.Generator().manual_seed(4)
    A = torch.randn(40, 90, dtype=dt, generator=g)
    Ah = ops.as_colmajor(A.clone())
    th = torch.zeros(40, dtype=dt)
    ops.gelqf(Ah, th)
    Ad = ops.as_colmajor(A.clone()).cuda()
    Ad = ops.as_colmajor(Ad)
    td = torch.zeros(40, dtype=dt, device="cuda")
    ops.gelqf(Ad, td)
    assert torch.allclose(torch.tril(Ad.cpu()), torch.tril(Ah), atol=1e-12)
    assert torch.allclose(td.cpu(), th, atol=1e-12)


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 130, 200, 448, 500, 512])
@pytest.mark.parametrize("variant", [0, 1])
def test_potrf_tile_variants(n, variant):
    """Both fp64 tile Cholesky kernels (0 = one-CU potrf_lds, 1 = the
    multi-workgroup 64-blocked potrf_mc) against the fp64 torch reference;
    lda > n, upper triangle untouched."""
    from slate_amd import _native
    X = ref(cm(n, n, torch.float64, 77))
    S = X @ X.mT + n * torch.eye(n, dtype=torch.float64, device="cuda")
    Abig = _cm(torch.zeros(n + 9, n, dtype=torch.float64, device="cuda"), "cuda")
    Abig[:n].copy_(S)
    A = Abig[:n]
    info = torch.zeros(1, dtype=torch.int64, device="cuda")
    _native.hip().potrf_tile_variant(variant, n, A.data_ptr(), A.stride(1), info.data_ptr(),
                                     torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert int(info.item()) == 0
    L = torch.tril(A)
    Lr = torch.linalg.cholesky(S)
    assert (L - Lr).abs().max() / Lr.abs().max() < 1e-13
    assert (torch.triu(A, 1) == torch.triu(S, 1)).all()


@pytest.mark.parametrize("bad", [0, 1, 62, 63, 64, 65, 127, 300, 511])
def test_potrf_mc_info(bad):
    from slate_amd import _native
    n = 512
    S = 4.0 * torch.eye(n, dtype=torch.float64, device="cuda")
    S[bad, bad] = -1.0
    if bad + 3 < n:
        S[bad + 3, bad + 3] = -2.0          # a later failure must not win
    A = _cm(S, "cuda")
    info = torch.zeros(1, dtype=torch.int64, device="cuda")
    _native.hip().potrf_tile_variant(1, n, A.data_ptr(), A.stride(1), info.data_ptr(),
                                     torch.cuda.current_stream().cuda_stream)
    assert int(info.item()) == bad + 1
