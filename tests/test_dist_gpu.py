"""GPU tests of the distributed-driver machinery on one MI355X.

* the device row-exchange kernels (swap plan, owner-masked pack/unpack,
  tournament selection -> LAPACK ipiv) against their host twins;
* the getrf driver (partial pivoting with lookahead 0/1/2, CALU, no
  pivoting) on the GPU;
* multi-rank rehearsals: 2 and 4 ranks sharing cuda:0 over gloo (RCCL
  refuses two ranks on one GPU), running the same stream/event pipelines,
  device kernels and collectives call pattern as the 8-GPU node.
"""
import pytest
import torch

import slate_amd as sl
from slate_amd import ops
from slate_amd.core.enums import MethodLU, Option, Uplo

from dist_util import run_dist

pytestmark = pytest.mark.gpu


def _rand_pivots(ns, m, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.tensor([int(torch.randint(i, m, (1,), generator=g)) for i in range(ns)], dtype=torch.int64)


def _plan(plan):
    nt = int(plan[0].item() & 0xFFFFFFFF)
    return nt, plan[1:1 + nt].tolist(), plan[1025:1025 + nt].tolist()


@pytest.mark.parametrize("ns,m,r0,incx", [(16, 200, 0, 1), (512, 4000, 1024, 1), (300, 1300, 512, -1)])
def test_swap_plan_device_equals_host(ns, m, r0, incx):
    # fixed-slot layout: window row q in slot q, the row swap q leaves below
    # the window in slot ns + q (-1: none) -- identical on every rank and on
    # host and device (the distributed exchange sums slot-wise)
    rel = _rand_pivots(ns, m - r0, 7)
    ipiv = torch.zeros(r0 + ns, dtype=torch.int64)
    ipiv[r0:] = rel                              # panel-relative, like getrf
    hp = ops.swap_plan(ipiv, r0, r0 + ns, ioff=-r0, incx=incx)
    for _ in range(3):                           # and run to run
        dp = ops.swap_plan(ipiv.cuda(), r0, r0 + ns, ioff=-r0, incx=incx)
        torch.cuda.synchronize()
        assert _plan(dp.cpu()) == _plan(hp)


@pytest.mark.parametrize("dt", [torch.float64, torch.complex64])
@pytest.mark.parametrize("p", [1, 2, 3])
def test_xchg_gather_scatter_device_equals_host(dt, p):
    nb, m, ncol, kb, r0 = 32, 600, 37, 32, 64
    ipiv = torch.zeros(r0 + kb, dtype=torch.int64)
    ipiv[r0:] = _rand_pivots(kb, m - r0, 3)
    from slate_amd.core.storage import numroc
    for pr in range(p):
        mloc = numroc(m, nb, pr, p)
        A = torch.randn(ncol, mloc, dtype=dt).t()
        X = ops.colmajor_empty(2 * kb, ncol, dt, "cpu")
        hp = ops.swap_plan(ipiv, r0, r0 + kb, ioff=-r0)
        ops.xchg_gather(hp, A, X, nb, p, pr)
        Ad = A.cuda().t().contiguous().t()
        Xd = ops.colmajor_empty(2 * kb, ncol, dt, "cuda")
        dp = ops.swap_plan(ipiv.cuda(), r0, r0 + kb, ioff=-r0)
        ops.xchg_gather(dp, Ad, Xd, nb, p, pr)
        torch.cuda.synchronize()
        torch.testing.assert_close(Xd.cpu(), X, rtol=0, atol=0)
        B = A.clone()
        ops.xchg_scatter(hp, X, B, nb, p, pr)
        Bd = Ad.clone()
        ops.xchg_scatter(dp, Xd, Bd, nb, p, pr)
        torch.cuda.synchronize()
        torch.testing.assert_close(Bd.cpu(), B, rtol=0, atol=0)


@pytest.mark.parametrize("kb,r0", [(8, 0), (512, 4096), (100, 300)])
def test_sel_to_ipiv_device_equals_host(kb, r0):
    g = torch.Generator().manual_seed(kb)
    sel = torch.randperm(4 * kb, generator=g)[:kb] + r0
    h = torch.zeros(kb, dtype=torch.int64)
    ops.sel_to_ipiv(sel, r0, h)
    d = torch.zeros(kb, dtype=torch.int64, device="cuda")
    ops.sel_to_ipiv(sel.cuda(), r0, d)
    torch.cuda.synchronize()
    assert torch.equal(d.cpu(), h)
    # the swap sequence brings exactly sel[i] to row r0 + i
    rows = list(range(5 * kb + r0))
    for i, pv in enumerate(h.tolist()):
        a, b = r0 + i, r0 + pv
        rows[a], rows[b] = rows[b], rows[a]
    assert rows[r0:r0 + kb] == sel.tolist()


def _gpu_mat(m, n, nb, seed, p=1, q=1):
    A = sl.Matrix(m, n, nb=nb, p=p, q=q, device="cuda")
    A.insertLocalTiles(device=0)
    sl.generate_matrix(A, "rands", seed)
    return A


def _lu_residual(A0, F, piv, n):
    L = torch.tril(F, -1) + torch.eye(n, dtype=F.dtype, device=F.device)
    PA = A0.clone()
    perm = list(range(n))
    for i, pv in enumerate(piv.ipiv.tolist()):
        perm[i], perm[pv] = perm[pv], perm[i]
    PA = A0[torch.as_tensor(perm, device=A0.device)]
    return ((L @ torch.triu(F) - PA).norm() / A0.norm()).item(), L


@pytest.mark.parametrize("la", [0, 1, 2])
def test_getrf_driver_lookahead_gpu(la):
    n, nb = 3072, 256
    A = _gpu_mat(n, n, nb, 41)
    A0 = A.storage.local[A.storage.origin_slot][:n, :n].clone()
    piv = sl.Pivots()
    assert sl.getrf(A, piv, {Option.Lookahead: la}) == 0
    torch.cuda.synchronize()
    F = A.storage.local[A.storage.origin_slot][:n, :n]
    r, L = _lu_residual(A0, F, piv, n)
    assert r < 64 * 2.2e-16 * n ** 0.5 * 4, r
    assert L.abs().max().item() <= 1.0 + 1e-12


def test_getrf_calu_gpu():
    import os
    n, nb = 2048, 256
    os.environ["SLATE_AMD_CALU_LEAF"] = "512"
    try:
        A = _gpu_mat(n, n, nb, 42)
        A0 = A.storage.local[A.storage.origin_slot][:n, :n].clone()
        piv = sl.Pivots()
        assert sl.getrf(A, piv, {Option.MethodLU: MethodLU.CALU}) == 0
        torch.cuda.synchronize()
    finally:
        del os.environ["SLATE_AMD_CALU_LEAF"]
    F = A.storage.local[A.storage.origin_slot][:n, :n]
    r, L = _lu_residual(A0, F, piv, n)
    assert r < 1e-12, r
    assert L.abs().max().item() < 20.0        # tournament growth stays small


# ------------------------------------------------- multi-rank on one GPU
def _check_grid_gpu(rank, size, p, q):
    import os
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from slate_amd.models.aux import allgather_dense as D
    n, nb = 1024, 128
    from slate_amd.parallel import comm as comm_mod

    def one_stream_per_comm(fn):
        """every communicator is driven from ONE stream
        inside a driver (sync RCCL collectives run on the issuing stream)."""
        comm_mod.STREAM_LOG["used"].clear()
        comm_mod.STREAM_LOG["on"] = True
        try:
            out = fn()
        finally:
            comm_mod.STREAM_LOG["on"] = False
        bad = {k: v for k, v in comm_mod.STREAM_LOG["used"].items() if len(v) > 1}
        assert not bad, bad
        return out
    # potrf
    A = sl.HermitianMatrix(Uplo.Lower, n, nb=nb, p=p, q=q, device=dev)
    A.insertLocalTiles(device=0)
    sl.generate_matrix(A, "poev", 3)
    Af = D(A)
    Af = torch.tril(Af) + torch.tril(Af, -1).mT
    assert one_stream_per_comm(lambda: sl.potrf(A, {Option.Lookahead: 1})) == 0
    L = torch.tril(D(A))
    assert ((L @ L.mT - Af).norm() / Af.norm()).item() < 1e-14
    # getrf: partial pivoting (lookahead 2; rows-on-owners panel, then the
    # all-gather form) and CALU
    for opts, gather in (({Option.Lookahead: 2}, "0"), ({Option.Lookahead: 2}, "1"),
                         ({Option.MethodLU: MethodLU.CALU}, "0")):
        os.environ["SLATE_AMD_CALU_LEAF"] = "256"
        os.environ["SLATE_AMD_LU_PANEL_GATHER"] = gather
        A = sl.Matrix(n, n, nb=nb, p=p, q=q, device=dev)
        A.insertLocalTiles(device=0)
        sl.generate_matrix(A, "rands", 4)
        A0 = D(A)
        piv = sl.Pivots()
        assert one_stream_per_comm(lambda: sl.getrf(A, piv, opts)) == 0
        r, _ = _lu_residual(A0, D(A), piv, n)
        assert r < 1e-12, (opts, r)
    os.environ["SLATE_AMD_LU_PANEL_GATHER"] = "0"
    # geqrf
    A = sl.Matrix(2 * n, n // 2, nb=nb, p=p, q=q, device=dev)
    A.insertLocalTiles(device=0)
    sl.generate_matrix(A, "rands", 5)
    A0 = D(A)
    T = sl.TriangularFactors()
    sl.geqrf(A, T)
    R = torch.triu(D(A)[: n // 2])
    assert ((R.mT @ R - A0.mT @ A0).norm() / (A0.norm() ** 2)).item() < 1e-14
    # heev: he2hb on the grid, band to rank 0, grid back-transforms
    m = 384
    H = sl.HermitianMatrix(Uplo.Lower, m, nb=64, p=p, q=q, device=dev)
    H.insertLocalTiles(device=0)
    sl.generate_matrix(H, "rands", 6)
    Hf = D(H)
    Hf = torch.tril(Hf) + torch.tril(Hf, -1).mT
    Z = sl.Matrix(m, m, nb=64, p=p, q=q, device=dev)
    Z.insertLocalTiles(device=0)
    w = sl.heev(H, None, Z)
    Zd = D(Z)
    w = w.to(Zd.device)
    assert ((Hf @ Zd - Zd * w).abs().max() / (Hf.abs().max() * m)).item() < 1e-13
    # svd: ge2tb on the grid (QR + LQ panels), tb2bd on rank 0, bdsqr by rows
    G = sl.Matrix(320, 200, nb=64, p=p, q=q, device=dev)
    G.insertLocalTiles(device=0)
    sl.generate_matrix(G, "rands", 7)
    G0 = D(G)
    U = sl.Matrix(320, 200, nb=64, p=p, q=q, device=dev)
    U.insertLocalTiles(device=0)
    VH = sl.Matrix(200, 200, nb=64, p=p, q=q, device=dev)
    VH.insertLocalTiles(device=0)
    s = sl.svd(G, None, U, VH, {Option.InnerBlocking: 32}).to(dev)
    assert ((D(U) @ torch.diag(s) @ D(VH) - G0).abs().max() / (G0.abs().max() * 320)).item() < 1e-13
    assert ((s.cpu() - torch.linalg.svdvals(G0.cpu())).abs().max() / s.max().cpu()).item() < 1e-13


@pytest.mark.parametrize("grid", [(2, 1), (1, 2), (2, 2)], ids=lambda g: f"{g[0]}x{g[1]}")
def test_multirank_one_gpu(grid):
    run_dist(_check_grid_gpu, grid[0] * grid[1], *grid, timeout=240)


def _check_lu_peer(rank, size, p, q, n=1024):
    """The device-resident panel (peer-mapped mailboxes, one persistent launch
    per 32-column block) against the host-issued record all-gather: the
    same pivots and bit-identical factors, and no per-column collective.
    n = 4096 on 2x1 gives each rank more than 1024 panel rows, so the panel
    runs G > 1 workgroups per rank and the leader's arg-max over their
    partials is exercised (the winner's candidate row)."""
    import os
    from slate_amd.models import lu as lu_mod
    from slate_amd.models.aux import allgather_dense as D
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    nb = 256
    os.environ["SLATE_AMD_LU_PANEL_GATHER"] = "0"
    out = {}
    for mode in ("0", "1"):
        os.environ["SLATE_AMD_LU_PEER"] = mode
        for k in lu_mod.LU_DIST_STATS:
            lu_mod.LU_DIST_STATS[k] = 0
        A = sl.Matrix(n, n, nb=nb, p=p, q=q, device=dev)
        A.insertLocalTiles(device=0)
        sl.generate_matrix(A, "rands", 11)
        A0 = D(A)
        piv = sl.Pivots()
        assert sl.getrf(A, piv, {Option.Lookahead: 1}) == 0
        torch.cuda.synchronize()
        r, L = _lu_residual(A0, D(A), piv, n)
        assert r < 1e-12 and L.abs().max().item() <= 1.0 + 1e-12, (mode, r)
        out[mode] = (A.storage.local[A.storage.origin_slot].clone(), piv.ipiv.clone(), dict(lu_mod.LU_DIST_STATS))
    os.environ["SLATE_AMD_LU_PEER"] = "1"
    f0, p0, st0 = out["0"]
    f1, p1, st1 = out["1"]
    assert torch.equal(p0.cpu(), p1.cpu())
    assert torch.equal(f0, f1), (f0 - f1).abs().max().item()
    panels = n // nb
    # host-issued form: one record all-gather per panel column
    assert st0["record_allgathers"] == st0["columns"] > 0, st0
    # device form: no per-column collective, kb / 32 launches per panel
    assert st1["record_allgathers"] == 0 and st1["columns"] == st0["columns"], st1
    assert st1["base_launches"] <= panels * (nb // 32), st1
    print(f"rank {rank}: peer LU stats {st1} (host form {st0})")


@pytest.mark.parametrize("grid,n", [((2, 1), 1024), ((2, 2), 1024), ((2, 1), 4096)],
                         ids=lambda g: f"{g[0]}x{g[1]}" if isinstance(g, tuple) else f"n{g}")
def test_lu_panel_peer_mailbox(grid, n):
    run_dist(_check_lu_peer, grid[0] * grid[1], *grid, n, timeout=240)
