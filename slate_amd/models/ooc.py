"""Out-of-core LU and QR for a host-resident matrix factored on the GPU.

Reference: SLATE's host-origin / device-target workspace streaming
(include/slate/BaseMatrix.hh:2640-2781 tileGetForReading/Writing and
release, 3878-3972 releaseWorkspace): tiles visit the device on demand and
leave after their last use, so the matrix need not fit in device memory.
models/chol_ooc.py is the Cholesky member of this family.

MI355X design (one rank, origin Host, Target.Devices, matrix larger than the
device budget or SLATE_AMD_OOC_COLS forced): left-looking by block columns
of W columns (a multiple of nb).  For block column J (columns J0 : J0+w):

  P <- A[:, J]                                    host -> device
  for each finished block column K < J (streamed on a copy stream, the next
  one in flight while the current one's GEMMs run):
      LU:  P[K rows] = L_KK^{-1} P[K rows];  P[below] -= L_K P[K rows]
      QR:  P[K0:] = Q_K^H P[K0:]   (the block's per-panel reflectors, T on device)
  factor P[J0:, :] in core (the one-rank getrf / geqrf pipelines)
  A[:, J] <- P                                    device -> host

Partial pivoting without re-touching the host: a finished LU block column
is stored in the row order current when it was factored; later blocks only
interchange rows below it, so when block K is streamed for block J its L
rows are re-ordered on the device by one row gather (index = the stored
order's inverse composed with the current order, built on the host in
O(m)).  One closing pass brings every stored block to the final order.

Device memory: four m x W buffers (panel, gather target, two streaming
buffers).  Host <-> device traffic O(m n^2 / W) words, overlapped with the
GEMMs.  With 288 GB of HBM3E per MI355X this is the path for local blocks
above ~190 000^2 (fp64).
"""
from __future__ import annotations

import numpy as np
import torch

from .. import ops
from ..utils.trace import trace_block
from .chol_ooc import device_budget


def ooc_block_columns(m, n, nb, dt, dev, nbufs):
    """Block-column width W (a multiple of nb) or 0 when the m x n matrix
    fits the device budget (in-core path)."""
    import os
    forced = os.environ.get("SLATE_AMD_OOC_COLS")
    es = torch.empty(0, dtype=dt).element_size()
    if forced:
        return max(nb, int(forced) // nb * nb)
    budget = device_budget(dev)
    if m * n * es <= budget:
        return 0
    return max(nb, budget // (nbufs * max(m, 1) * es) // nb * nb)


def ooc_applicable(A, s, slot):
    """One rank, host origin, device target, whole matrix (not a view)."""
    from ..core.storage import DEV, HOST
    bc = s.bc
    return (slot == DEV and s.origin_slot == HOST and bc.p * bc.q == 1 and not A.ioffset and not A.joffset
            and not A.row0_offset and not A.col0_offset and A.m() == s.m and A.n() == s.n
            and torch.cuda.is_available())


class _Streamer:
    """Double-buffered host -> device fetches of block columns on a copy
    stream; a buffer is refilled only after the compute stream is done
    with it."""

    def __init__(self, m, W, dt, dev, pinned):
        self.bufs = [ops.colmajor_empty(m, W, dt, dev) for _ in range(2)]
        self.cs = torch.cuda.Stream(device=dev)
        self.cur = torch.cuda.current_stream(dev)
        self.pinned = pinned
        self.ev = {}

    def fetch(self, src, slot, key):
        r, c = src.shape
        B = self.bufs[slot][:r, :c]
        with torch.cuda.stream(self.cs):
            self.cs.wait_stream(self.cur)
            B.copy_(src, non_blocking=self.pinned)
            ev = torch.cuda.Event()
            ev.record(self.cs)
        self.ev[key] = ev
        return B

    def ready(self, key):
        self.cur.wait_event(self.ev.pop(key))


def _idx(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.int64)).to(dev)


def getrf_ooc(H, m, n, nb, W, dev, thr=1.0, la=1):
    """P A = L U of the host column-major m x n matrix H in place with block
    columns of W columns on ``dev``.  Returns (info, ipiv): ipiv the global
    0-based pivot rows (LAPACK order), info the first zero pivot (1-based)."""
    from ..core.enums import Option
    from ..core.matrix import Matrix, Pivots
    from ..parallel.comm import self_comm
    from .lu import getrf as _getrf
    dt = H.dtype
    kmax = min(m, n)
    st = _Streamer(m, W, dt, dev, H.is_pinned())
    cur = st.cur
    panel = ops.colmajor_empty(m, W, dt, dev)
    gath = ops.colmajor_empty(m, W, dt, dev)
    perm = np.arange(m, dtype=np.int64)      # position i holds original row perm[i]
    inv_of = {}                              # block J0 -> inverse of its stored row order
    ipiv = []
    info = 0
    with trace_block("getrf_ooc"):
        for J0 in range(0, n, W):
            w = min(W, n - J0)
            P = panel[:, :w]
            # unfactored columns are still in the original row order
            raw = gath[:, :w]
            raw.copy_(H[:, J0:J0 + w], non_blocking=st.pinned)
            ops.row_gather(raw, P, _idx(perm, dev))
            Ks = [K0 for K0 in range(0, min(J0, kmax), W)]
            if Ks:
                st.fetch(H[Ks[0]:, Ks[0]:Ks[0] + min(W, kmax - Ks[0])], 0, Ks[0])
            for i, K0 in enumerate(Ks):
                if i + 1 < len(Ks):
                    K1 = Ks[i + 1]
                    st.fetch(H[K1:, K1:K1 + min(W, kmax - K1)], (i + 1) % 2, K1)
                st.ready(K0)
                kw = min(W, kmax - K0)
                B = st.bufs[i % 2][:m - K0, :kw]
                with trace_block("getrf_ooc::update"):
                    ops.trsm('L', 'L', 'N', 'U', 1.0, B[:kw], P[K0:K0 + kw])
                    r1 = K0 + kw
                    if m > r1:
                        g = inv_of[K0][perm[r1:]] - K0          # stored row of each current row
                        if np.array_equal(g, np.arange(kw, m - K0)):
                            L = B[kw:]
                        else:
                            L = gath[:m - r1, :kw]
                            ops.row_gather(B, L, _idx(g, dev))
                        ops.gemm(-1.0, L, P[K0:K0 + kw], 1.0, P[r1:])
            if J0 < kmax:
                with trace_block("getrf_ooc::panel"):
                    mq = m - J0
                    Q = P[J0:]
                    M = Matrix.fromLAPACK(mq, w, Q, max(1, panel.stride(1)), nb=nb, comm=self_comm())
                    pv = Pivots(nb)
                    inf = _getrf(M, pv, {Option.Lookahead: la, Option.PivotThreshold: thr})
                    loc = pv.ipiv.numpy()
                    if inf and not info:
                        info = J0 + inf
                    for t, r in enumerate(loc.tolist()):
                        a, b = J0 + t, J0 + r
                        if a != b:
                            perm[a], perm[b] = perm[b], perm[a]
                    ipiv.append(loc + J0)
                inv = np.empty(m, dtype=np.int64)
                inv[perm] = np.arange(m, dtype=np.int64)
                inv_of[J0] = inv
            H[:, J0:J0 + w].copy_(P, non_blocking=st.pinned)
        # closing pass: stored L rows into the final row order
        with trace_block("getrf_ooc::reorder"):
            for K0 in range(0, kmax, W):
                kw = min(W, kmax - K0)
                r1 = K0 + kw
                if m <= r1:
                    continue
                g = inv_of[K0][perm[r1:]] - r1
                if np.array_equal(g, np.arange(m - r1)):
                    continue
                B = panel[:m - r1, :kw]
                B.copy_(H[r1:, K0:K0 + kw], non_blocking=st.pinned)
                L = gath[:m - r1, :kw]
                ops.row_gather(B, L, _idx(g, dev))
                H[r1:, K0:K0 + kw].copy_(L, non_blocking=st.pinned)
        cur.synchronize()
    piv = torch.from_numpy(np.concatenate(ipiv)) if ipiv else torch.zeros(0, dtype=torch.int64)
    return info, piv


def geqrf_ooc(H, m, n, nb, W, dev, la=1):
    """A = Q R of the host column-major m x n matrix H in place with block
    columns of W columns on ``dev``.  Returns the per-panel factor list (the
    entries models/qr.py's unmqr consumes, T on the device)."""
    from ..core.enums import Option
    from ..core.matrix import Matrix, TriangularFactors
    from ..parallel.comm import self_comm
    from .qr import _apply_qh, geqrf as _geqrf
    dt = H.dtype
    kmax = min(m, n)
    st = _Streamer(m, W, dt, dev, H.is_pinned())
    cur = st.cur
    panel = ops.colmajor_empty(m, W, dt, dev)
    Vbuf = ops.colmajor_empty(m, nb, dt, dev)
    fac = []
    with trace_block("geqrf_ooc"):
        for J0 in range(0, n, W):
            w = min(W, n - J0)
            P = panel[:, :w]
            P.copy_(H[:, J0:J0 + w], non_blocking=st.pinned)
            Ks = [K0 for K0 in range(0, min(J0, kmax), W)]
            if Ks:
                st.fetch(H[Ks[0]:, Ks[0]:Ks[0] + min(W, kmax - Ks[0])], 0, Ks[0])
            for i, K0 in enumerate(Ks):
                if i + 1 < len(Ks):
                    K1 = Ks[i + 1]
                    st.fetch(H[K1:, K1:K1 + min(W, kmax - K1)], (i + 1) % 2, K1)
                st.ready(K0)
                B = st.bufs[i % 2][:m - K0, :min(W, kmax - K0)]
                with trace_block("geqrf_ooc::update"):
                    for f in fac:
                        r0, kb = f["r0"], f["kb"]
                        if r0 < K0 or r0 >= K0 + W:
                            continue
                        lr = r0 - K0
                        V = Vbuf[:m - r0, :kb]
                        ops.v_explicit(B[lr:, lr:lr + kb], V)
                        _apply_qh(V, f["T"], P[r0:])
            if J0 < kmax:
                with trace_block("geqrf_ooc::panel"):
                    M = Matrix.fromLAPACK(m - J0, w, P[J0:], max(1, panel.stride(1)), nb=nb, comm=self_comm())
                    TF = TriangularFactors()
                    _geqrf(M, TF, {Option.Lookahead: la})
                    for f in TF:
                        g = dict(f)
                        g["r0"] = J0 + f["r0"]
                        fac.append(g)
            H[:, J0:J0 + w].copy_(P, non_blocking=st.pinned)
        cur.synchronize()
    return fac
