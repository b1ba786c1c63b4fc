"""Loopback transport (parallel/comm.py LoopbackComm): one process plays rank
r of a p x q job; every collective becomes a same-size local copy and is
logged.  CPU checks: the drivers run to completion at every rank position,
the log holds the broadcasts the 2D algorithms need, and a 1-rank loopback
world gives the ordinary single-rank result."""
import pytest
import torch

import slate_amd as sl
from slate_amd.parallel import comm as C


@pytest.fixture(autouse=True)
def _restore_world():
    yield
    C._WORLD = None
    C.ProcessGrid._cache.clear()
    C.LoopbackComm.LOG.clear()


@pytest.mark.parametrize("grid,rank", [((2, 4), 0), ((2, 4), 7), ((4, 2), 5), ((1, 8), 3)])
def test_loopback_potrf_gemm_run_at_every_rank(grid, rank):
    p, q = grid
    C.loopback(p * q, rank)
    C.LoopbackComm.LOG.clear()
    n, nb = 384, 64
    A = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb, p=p, q=q)
    A.insertLocalTiles()
    sl.generate_matrix(A, "poev", seed=3)
    sl.potrf(A)
    ops = {(op, size) for op, size, _, _ in C.LoopbackComm.LOG}
    if q > 1:
        assert ("bcast", q) in ops          # panel rows along the process row
    if p > 1:
        assert ("bcast", p) in ops          # diagonal tile down the process column
    C.LoopbackComm.LOG.clear()
    X = sl.Matrix(n, n, nb=nb, p=p, q=q)
    X.insertLocalTiles()
    Y = sl.Matrix(n, n, nb=nb, p=p, q=q)
    Y.insertLocalTiles()
    Z = sl.Matrix(n, n, nb=nb, p=p, q=q)
    Z.insertLocalTiles()
    sl.gemm(1.0, X, Y, 0.0, Z)
    nbytes = sum(b for _, _, b, _ in C.LoopbackComm.LOG)
    # SUMMA: every k block travels along the row and down the column
    bc = X.storage.bc
    expect = 0
    if q > 1:
        expect += bc.mloc * n * 8
    if p > 1:
        expect += n * bc.nloc * 8
    assert nbytes == expect


def test_loopback_single_rank_matches_plain():
    n, nb = 256, 64
    A = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb)
    A.insertLocalTiles()
    sl.generate_matrix(A, "poev", seed=5)
    ref = A.storage.local[A.storage.origin_slot].clone()
    sl.potrf(A)
    want = A.storage.local[A.storage.origin_slot].clone()
    C.loopback(1, 0)
    B = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb)
    B.insertLocalTiles()
    B.storage.local[B.storage.origin_slot].copy_(ref)
    B.storage.mark_local_modified(B.storage.origin_slot)
    sl.potrf(B)
    got = B.storage.local[B.storage.origin_slot]
    assert torch.equal(torch.tril(got), torch.tril(want))


@pytest.mark.gpu
def test_loopback_link_model_holds_stream(monkeypatch):
    """SLATE_AMD_LOOPBACK_LINK: a bcast holds its issuing stream for
    alpha + bytes / beta (the spin kernel, aux.hip spin_ticks_kernel)."""
    monkeypatch.setenv("SLATE_AMD_LOOPBACK_LINK", "100,1")      # 100 us + 1 GB/s
    C.LoopbackComm._link = None
    try:
        comm = C.LoopbackComm(2, 1)
        t = torch.zeros(1 << 17, dtype=torch.float64, device="cuda")     # 1 MiB -> ~1.05 ms + 0.1
        comm.bcast(t, 0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        comm.bcast(t, 0)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        assert 1.1 < ms < 2.0, ms
    finally:
        C.LoopbackComm._link = None


def test_loopback_refuses_pivoted_getrf():
    """Pivoted LU needs the peers' pivot data: under the loopback transport
    it raises instead of running a row exchange planned from this rank's own
    bytes (which indexed past the local block on the GPU)."""
    C.loopback(8, 0)
    A = sl.Matrix(256, 256, nb=64, p=2, q=4)
    A.insertLocalTiles()
    with pytest.raises(sl.SlateError):
        sl.getrf(A, sl.Pivots())
