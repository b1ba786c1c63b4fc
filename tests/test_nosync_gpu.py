"""The factorization loops never wait for the GPU.

potrf / getrf / geqrf run under ``torch.cuda.set_sync_debug_mode("error")``:
any synchronising torch operation inside a driver (a pageable host->device
copy, ``.item()``, ``.cpu()``, ``nonzero``) raises.  The one wait a driver
does -- the info values at its end -- goes through a pinned non-blocking copy
and an event wait (``models/_util.read_to_host``), which is not such an op.
The CholeskyQR panel's fallback decision is taken on the device
(csrc/hip/qr_fast.hip), so the tall-QR case covers it too.

The multi-rank case is covered on the CPU (gloo stages every collective
through host memory by construction, so it cannot run under this mode)."""
import os

import pytest
import torch

import slate_amd as sl

pytestmark = pytest.mark.gpu


def _run_nosync(fn):
    torch.cuda.synchronize()
    old = torch.cuda.get_sync_debug_mode()
    torch.cuda.set_sync_debug_mode("error")
    try:
        return fn()
    finally:
        torch.cuda.set_sync_debug_mode(old)
        torch.cuda.synchronize()


@pytest.mark.parametrize("group", ["2", "1"])
def test_potrf_no_host_sync(group, monkeypatch):
    monkeypatch.setenv("SLATE_AMD_POTRF_GROUP", group)
    dev = torch.device("cuda")
    n, nb = 2048, 256
    A = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb, device=dev)
    A.insertLocalTiles(device=dev)
    sl.generate_matrix(A, "poev", seed=3)
    F0 = A.storage.local[A.storage.origin_slot][:n, :n].clone()
    info = _run_nosync(lambda: sl.potrf(A, {sl.Option.Lookahead: 1}))
    assert info == 0
    L = torch.tril(A.storage.local[A.storage.origin_slot][:n, :n])
    S = torch.tril(F0) + torch.tril(F0, -1).mT
    assert ((L @ L.mT - S).norm() / S.norm()).item() < 1e-14


def test_getrf_no_host_sync():
    dev = torch.device("cuda")
    n, nb = 2048, 256
    A = sl.Matrix(n, n, nb=nb, device=dev)
    A.insertLocalTiles(device=dev)
    sl.generate_matrix(A, "rands", seed=4)
    F0 = A.storage.local[A.storage.origin_slot][:n, :n].clone()
    piv = sl.Pivots()
    info = _run_nosync(lambda: sl.getrf(A, piv, {sl.Option.Lookahead: 2}))
    assert info == 0
    F = A.storage.local[A.storage.origin_slot][:n, :n]
    L = torch.tril(F, -1) + torch.eye(n, dtype=F.dtype, device=dev)
    U = torch.triu(F)
    perm = list(range(n))
    for i, j in enumerate(piv.ipiv.tolist()):
        perm[i], perm[j] = perm[j], perm[i]
    PA = F0[torch.as_tensor(perm, device=dev)]
    assert ((L @ U - PA).norm() / F0.norm()).item() < 1e-13


@pytest.mark.parametrize("mn", [(4096, 1024), (16384, 512)])
def test_geqrf_no_host_sync(mn):
    m, n = mn
    dev = torch.device("cuda")
    nb = 256 if n > 512 else 128
    A = sl.Matrix(m, n, nb=nb, device=dev)
    A.insertLocalTiles(device=dev)
    sl.generate_matrix(A, "rands", seed=5)
    F0 = A.storage.local[A.storage.origin_slot][:m, :n].clone()
    T = sl.TriangularFactors()
    info = _run_nosync(lambda: sl.geqrf(A, T))
    assert info == 0
    R = torch.triu(A.storage.local[A.storage.origin_slot][:n, :n])
    assert ((R.mT @ R - F0.mT @ F0).norm() / F0.norm() ** 2).item() < 1e-14


@pytest.mark.parametrize("la", [1, 2])
def test_potrf_diag_first_matches_serial(la, monkeypatch):
    """Regression for the diag-first race: with la = 1
    the next diagonal tile was factored on the diag stream before step t-1's
    trailing update had written it.  Pipelined and fully serial
    (SLATE_AMD_SERIAL=1: every stream is the current stream) runs must agree
    to rounding, on a size where the trailing GEMMs are long."""
    monkeypatch.setenv("SLATE_AMD_POTRF_GROUP", "1")
    dev = torch.device("cuda")
    n, nb = 8192, 512

    def run():
        A = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb, device=dev)
        A.insertLocalTiles(device=dev)
        sl.generate_matrix(A, "poev", seed=9)
        assert sl.potrf(A, {sl.Option.Lookahead: la}) == 0
        torch.cuda.synchronize()
        return torch.tril(A.storage.local[A.storage.origin_slot][:n, :n]).clone()

    Lp = run()
    monkeypatch.setenv("SLATE_AMD_SERIAL", "1")
    Ls = run()
    assert ((Lp - Ls).abs().max() / Ls.abs().max()).item() < 1e-13


def test_stream_census():
    """Every pipeline shares one panel, one diag and one update stream per
    device: with the current stream at most 4 work streams, one per hardware
    queue of the box's default GPU_MAX_HW_QUEUES."""
    from slate_amd.parallel.streams import MAX_WORK_STREAMS, StreamSet
    dev = torch.device("cuda")
    n, nb = 1024, 256
    H = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb, device=dev)
    H.insertLocalTiles(device=dev)
    sl.generate_matrix(H, "poev", seed=1)
    assert sl.potrf(H) == 0
    A = sl.Matrix(n, n, nb=nb, device=dev)
    A.insertLocalTiles(device=dev)
    sl.generate_matrix(A, "rands", seed=2)
    assert sl.getrf(A, sl.Pivots()) == 0
    Q = sl.Matrix(4 * n, n // 2, nb=128, device=dev)
    Q.insertLocalTiles(device=dev)
    sl.generate_matrix(Q, "rands", seed=3)
    sl.geqrf(Q, sl.TriangularFactors())
    torch.cuda.synchronize()
    # process-wide: panel, diag and ONE update stream plus the caller's
    # stream -- at most the 4 hardware queues
    sets = [s for s in StreamSet._cache.values() if s.gpu and not s.serial]
    assert sets
    assert StreamSet.census(dev) <= MAX_WORK_STREAMS
    assert len(StreamSet.streams_of(dev)) <= MAX_WORK_STREAMS - 1
    for s in sets:
        s.check_census()
    # the live update stream carries the reservation of the last pipeline
    # (geqrf: none), not the first one's 32 CUs
    ups = {id(s.update[0]) for s in sets}
    assert len(ups) == 1
    assert sets[0]._sh["upd"][0] == 0
    # back to getrf: the stream is replaced again, results unchanged
    A2 = sl.Matrix(n, n, nb=nb, device=dev)
    A2.insertLocalTiles(device=dev)
    sl.generate_matrix(A2, "rands", seed=2)
    assert sl.getrf(A2, sl.Pivots()) == 0
    torch.cuda.synchronize()
    assert StreamSet.census(dev) <= MAX_WORK_STREAMS
    assert torch.equal(A.storage.local[A.storage.origin_slot], A2.storage.local[A2.storage.origin_slot])


def test_retired_update_stream_outlives_its_tensors():
    """a tensor that recorded the CU-masked update stream
    (getrf's) and outlives the driver is freed after geqrf switched the live
    update stream to another reservation: the retired stream is parked, not
    destroyed, so the allocator's free-time event record is valid; getrf
    then gets the same parked stream back."""
    from slate_amd.parallel.streams import StreamSet
    dev = torch.device("cuda")
    n, nb = 1024, 256
    A = sl.Matrix(n, n, nb=nb, device=dev)
    A.insertLocalTiles(device=dev)
    sl.generate_matrix(A, "rands", seed=2)
    assert sl.getrf(A, sl.Pivots()) == 0
    sets = [s for s in StreamSet._cache.values() if s.gpu and not s.serial]
    masked = sets[0]._sh["upd"][1]
    keep = torch.empty(1 << 20, dtype=torch.float64, device=dev)
    with torch.cuda.stream(masked):
        keep.fill_(1.0)
    keep.record_stream(masked)
    Q = sl.Matrix(4 * n, n // 2, nb=128, device=dev)
    Q.insertLocalTiles(device=dev)
    sl.generate_matrix(Q, "rands", seed=3)
    T = sl.TriangularFactors()
    sl.geqrf(Q, T)
    assert sets[0]._sh["upd"][1] is not masked
    del keep                                  # event recorded on the parked stream
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    A2 = sl.Matrix(n, n, nb=nb, device=dev)
    A2.insertLocalTiles(device=dev)
    sl.generate_matrix(A2, "rands", seed=2)
    assert sl.getrf(A2, sl.Pivots()) == 0
    assert sets[0]._sh["upd"][1] is masked    # reused, not a new stream per switch
    del T
    torch.cuda.synchronize()


def test_potrf_use_graph():
    """Option.UseGraph: the one-rank potrf is captured once into a hipGraph
    and replayed; every replay on fresh input matches the eager factor and
    reports info through the graph's own info vector."""
    dev = torch.device("cuda")
    n, nb = 2048, 256
    A = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb, device=dev)
    A.insertLocalTiles(device=dev)
    buf = A.storage.local[A.storage.origin_slot]
    for seed in (3, 4, 5):
        sl.generate_matrix(A, "poev", seed=seed)
        F0 = buf[:n, :n].clone()
        assert sl.potrf(A, {sl.Option.Lookahead: 1, sl.Option.UseGraph: True}) == 0
        Lg = torch.tril(buf[:n, :n]).clone()
        buf[:n, :n].copy_(F0)
        assert sl.potrf(A, {sl.Option.Lookahead: 1}) == 0
        Le = torch.tril(buf[:n, :n])
        assert (Lg - Le).abs().max().item() <= 1e-12 * Le.abs().max().item()
    # a non-SPD input: info through the graph
    buf[:n, :n].copy_(F0)
    buf[100, 100] = -1.0
    assert sl.potrf(A, {sl.Option.Lookahead: 1, sl.Option.UseGraph: True}) == 101


def test_potrf_use_graph_workspace_survives_other_streams():
    """the captured kernels point into per-stream
    workspaces; the graph owns a private capture stream, so a larger eager
    potrf/trsm on fresh torch streams afterwards (which may be handed the
    pooled handles) cannot free them.  Capture, run bigger eager work on new
    streams, replay, compare."""
    dev = torch.device("cuda")
    n, nb = 2048, 256
    A = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb, device=dev)
    A.insertLocalTiles(device=dev)
    buf = A.storage.local[A.storage.origin_slot]
    sl.generate_matrix(A, "poev", seed=11)
    F0 = buf[:n, :n].clone()
    assert sl.potrf(A, {sl.Option.Lookahead: 1, sl.Option.UseGraph: True}) == 0
    from slate_amd import ops
    n2 = 3072
    B = sl.HermitianMatrix(sl.Uplo.Lower, n2, nb=512, device=dev)
    B.insertLocalTiles(device=dev)
    T = torch.eye(3000, dtype=torch.float64, device=dev).mT.contiguous().mT
    X = torch.randn(3000, 3000, dtype=torch.float64, device=dev).mT.contiguous().mT
    for _ in range(34):          # cycle through torch's round-robin stream pool
        st = torch.cuda.Stream(device=dev)
        with torch.cuda.stream(st):
            sl.generate_matrix(B, "poev", seed=12)
            assert sl.potrf(B, {sl.Option.Lookahead: 1}) == 0
            ops.trsm('L', 'L', 'N', 'N', 1.0, T, X)
        st.synchronize()
    buf[:n, :n].copy_(F0)
    assert sl.potrf(A, {sl.Option.Lookahead: 1, sl.Option.UseGraph: True}) == 0
    Lg = torch.tril(buf[:n, :n]).clone()
    buf[:n, :n].copy_(F0)
    assert sl.potrf(A, {sl.Option.Lookahead: 1}) == 0
    Le = torch.tril(buf[:n, :n])
    assert (Lg - Le).abs().max().item() <= 1e-12 * Le.abs().max().item()


@pytest.mark.parametrize("W", [512, 1536])
def test_potrf_out_of_core(W, monkeypatch):
    """Host-origin matrix, device target, forced out-of-core block columns
    (models/chol_ooc.py): same factor as the in-core path."""
    monkeypatch.setenv("SLATE_AMD_OOC_COLS", str(W))
    n, nb = 3000, 256
    A = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb)
    A.insertLocalTiles()                                # host origin
    sl.generate_matrix(A, "poev", seed=9)
    H = A.storage.local[A.storage.origin_slot]
    S0 = H[:n, :n].clone()
    assert sl.potrf(A, {sl.Option.Target: sl.Target.Devices}) == 0
    L = torch.tril(A.storage.local[A.storage.origin_slot][:n, :n])
    S = torch.tril(S0) + torch.tril(S0, -1).mT
    assert ((L @ L.mT - S).norm() / S.norm()).item() < 1e-14


@pytest.mark.parametrize("shape,W", [((3000, 3000), 512), ((3300, 2200), 768), ((1800, 2600), 512)],
                         ids=["sq", "tall", "wide"])
def test_getrf_out_of_core(shape, W, monkeypatch):
    """Host-origin LU with forced out-of-core block columns (models/ooc.py):
    the streamed left-looking factorization with deferred row re-ordering
    reproduces P A = L U, and its pivots drive getrs."""
    monkeypatch.setenv("SLATE_AMD_OOC_COLS", str(W))
    m, n = shape
    nb = 256
    A = sl.Matrix(m, n, nb=nb)
    A.insertLocalTiles()                                # host origin
    sl.generate_matrix(A, "rand", seed=5)
    H = A.storage.local[A.storage.origin_slot]
    A0 = H[:m, :n].clone()
    piv = sl.Pivots()
    assert sl.getrf(A, piv, {sl.Option.Target: sl.Target.Devices}) == 0
    F = A.storage.local[A.storage.origin_slot][:m, :n]
    k = min(m, n)
    L = torch.tril(F[:, :k], -1) + torch.eye(m, k, dtype=F.dtype)
    U = torch.triu(F[:k, :])
    PA = A0.clone()
    for i, r in enumerate(piv.ipiv.tolist()):
        if r != i:
            PA[[i, r]] = PA[[r, i]]
    assert ((L @ U - PA).norm() / A0.norm()).item() < 1e-14
    # the in-core factorization picks the same pivots
    monkeypatch.delenv("SLATE_AMD_OOC_COLS")
    B = sl.Matrix(m, n, nb=nb)
    B.insertLocalTiles()
    sl.generate_matrix(B, "rand", seed=5)
    piv2 = sl.Pivots()
    assert sl.getrf(B, piv2, {sl.Option.Target: sl.Target.Devices}) == 0
    assert torch.equal(piv.ipiv, piv2.ipiv)


@pytest.mark.parametrize("shape,W", [((3000, 2000), 512), ((2400, 2400), 768)], ids=["tall", "sq"])
def test_geqrf_out_of_core(shape, W, monkeypatch):
    """Host-origin QR with forced out-of-core block columns: R matches the
    in-core factor and unmqr with the streamed factors reproduces A."""
    monkeypatch.setenv("SLATE_AMD_OOC_COLS", str(W))
    m, n = shape
    nb = 256
    A = sl.Matrix(m, n, nb=nb)
    A.insertLocalTiles()
    sl.generate_matrix(A, "rand", seed=6)
    A0 = A.storage.local[A.storage.origin_slot][:m, :n].clone()
    T = sl.TriangularFactors()
    assert sl.geqrf(A, T, {sl.Option.Target: sl.Target.Devices}) == 0
    monkeypatch.delenv("SLATE_AMD_OOC_COLS")
    F = A.storage.local[A.storage.origin_slot][:m, :n].clone()
    R = torch.triu(F[:n, :])
    # Q R = A: apply Q to [R; 0] with the streamed factors
    C = sl.Matrix(m, n, nb=nb)
    C.insertLocalTiles()
    C.storage.local[C.storage.origin_slot][:m, :n].zero_()
    C.storage.local[C.storage.origin_slot][:n, :n].copy_(R)
    sl.unmqr(sl.Side.Left, sl.Op.NoTrans, A, T, C, {sl.Option.Target: sl.Target.Devices})
    QR = C.storage.local[C.storage.origin_slot][:m, :n]
    assert ((QR - A0).norm() / A0.norm()).item() < 1e-14
    # R agrees with the in-core factor up to row signs
    B = sl.Matrix(m, n, nb=nb)
    B.insertLocalTiles()
    sl.generate_matrix(B, "rand", seed=6)
    T2 = sl.TriangularFactors()
    sl.geqrf(B, T2, {sl.Option.Target: sl.Target.Devices})
    B.storage.sync_origin()                             # the in-core factor lives on the device
    R2 = torch.triu(B.storage.local[B.storage.origin_slot][:n, :n])
    assert ((R.abs() - R2.abs()).norm() / R2.norm()).item() < 1e-12
