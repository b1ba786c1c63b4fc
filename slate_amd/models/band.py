"""Band drivers: gbtrf / gbtrs / gbsv (band LU with partial pivoting),
pbtrf / pbtrs / pbsv (band Cholesky), tbsm (triangular band solve, with
the gbtrf pivots: tbsmPivots), gbmm, hbmm, band_mask.

Reference: `src/gbtrf.cc:20-348` (panel + band-limited trailing update,
upper bandwidth grows to kl + ku), `src/gbtrs.cc`, `src/gbsv.cc`,
`src/pbtrf.cc`, `src/pbtrs.cc`, `src/pbsv.cc`, `src/tbsm.cc`,
`src/tbsmPivots.cc`, `src/gbmm.cc`, `src/hbmm.cc`.

MI355X design on the compact band storage (core/band_storage.py: tile
columns 1-D cyclic over the ranks, each local tile column one contiguous
slab of its band tiles):

* factorizations: the panel of tile column k is ONE contiguous slab block
  on its owner (GPU LU with partial pivoting over the kb + kl rows that can
  be non-zero, or potrf + trsm); panel and pivots travel in one packed
  broadcast; every rank then updates ITS tile columns inside the window
  (k, k + KU] -- swaps, trsm and one MFMA GEMM per column, each on a
  contiguous slab sub-block (the rows shift by one tile per column, so the
  columns cannot share a launch).  The owner of column k + 1 updates it
  first, so its next panel overlaps the other ranks' updates.  Cost
  O(n kl (kl + ku)), memory O(n (kl + ku)).
* solves: the right-hand side stays 1-D row-cyclic over the ranks (tile
  row i with the owner of band column i); each step's window of kb +
  bandwidth rows is gathered point-to-point onto the owner of the factor
  column, solved / updated there and scattered back (_DistX) -- per-rank
  memory O(local rows + one window), never the replicated n x nrhs B.
* products: B and C move to 1-D row-cyclic work layouts matched to the
  band's column ownership (one redistribution each); each rank multiplies
  its slabs and the partial blocks travel point-to-point to the owners of
  their rows (op(A) = A), or the B tiles of each column's window travel to
  the column's owner (op(A) = A^T / A^H) -- no replication, no all-reduce.
"""
from __future__ import annotations

import torch

from .. import ops
from ..core.band_storage import BandStorage, tiles_for
from ..core.enums import Diag, Op, Side, Uplo
from ..core.exceptions import SlateError
from ..core.matrix import Pivots
from ..utils.trace import trace_block
from ._util import conj_trans

_LOWER_MASK = (1, 1 << 40, 1, 0, 1, 0, 0, 0, 0)      # element-level lower triangle of the output


def _is_band(A):
    return isinstance(A.storage, BandStorage)


def _bands(A):
    kl = A.lowerBandwidth() if hasattr(A, "lowerBandwidth") else A.m()
    ku = A.upperBandwidth() if hasattr(A, "upperBandwidth") else A.n()
    return kl, ku


def _need_band(A, who):
    if not _is_band(A):
        raise SlateError(f"{who}: needs a band matrix (BandMatrix / HermitianBandMatrix / TriangularBandMatrix)")
    if A.ioffset or A.joffset or A.row0_offset or A.col0_offset:
        raise SlateError(f"{who}: sub-matrix views of band matrices are not supported")


# ------------------------------------------------------------------ masks
def _zero_lower(t, s):
    """Zero the entries (a, b) of tile t with a - b >= s."""
    mb, nbt = t.shape
    if mb == 0 or nbt == 0 or s > mb - 1:
        return
    if s >= 0:
        ops.geset(0.0, 0.0, t[s:, :], uplo='L')
        return
    c = min(-s, nbt)
    ops.geset(0.0, 0.0, t[:, :c])
    if c < nbt:
        ops.geset(0.0, 0.0, t[:, c:], uplo='L')


def _zero_upper(t, s):
    """Zero the entries (a, b) of tile t with b - a >= s."""
    mb, nbt = t.shape
    if mb == 0 or nbt == 0 or s > nbt - 1:
        return
    if s >= 0:
        ops.geset(0.0, 0.0, t[:, s:], uplo='U')
        return
    r = min(-s, mb)
    ops.geset(0.0, 0.0, t[:r, :])
    if r < mb:
        ops.geset(0.0, 0.0, t[r:, :], uplo='U')


def band_mask(A, kl=None, ku=None):
    """Zero every stored entry outside -ku <= i - j <= kl (global indices)."""
    s = A.storage
    if kl is None:
        kl, ku = (A._kl, A._ku) if hasattr(A, "_kl") else _bands(A)
    if _is_band(A):
        slot = s.band_slot()
        for (i, j, sl) in list(s.tiles.keys()):
            if sl != slot or not s.tileIsLocal(i, j):
                continue
            t = s.tiles[(i, j, sl)]
            d = s.row_offsets[i] - s.col_offsets[j]
            _zero_lower(t, kl - d + 1)
            _zero_upper(t, ku + d + 1)
        s.mark_local_modified(slot)
        return A
    lb = A.local_block()
    if lb.mloc == 0 or lb.nloc == 0:
        return A
    dev = lb.data.device
    gr = torch.tensor([lb.global_row(i) for i in range(lb.mloc)], device=dev)
    gc = torch.tensor([lb.global_col(j) for j in range(lb.nloc)], device=dev)
    d = gr[:, None] - gc[None, :]
    lb.data.masked_fill_((d > kl) | (d < -ku), 0)
    s.mark_local_modified(s.origin_slot)
    return A


# ------------------------------------------------------------------ helpers
def _slab(A):
    s = A.storage
    slot = s.band_slot()
    return s, slot, s.sync_slab(slot)


def _col_block(s, buf, k, g_lo, g_hi):
    """Slab block of tile column k holding global rows [g_lo, g_hi)."""
    r = s.slab_row(g_lo, k)
    c = s.local_col(k)
    return buf[r:r + (g_hi - g_lo), c:c + s.tileNb(k)]


def _bcast_rows(comm, X, lo, hi, root):
    if comm.size == 1 or hi <= lo:
        return
    tmp = X[lo:hi].contiguous()
    comm.bcast(tmp, root)
    X[lo:hi].copy_(tmp)


def _cm_copy(D, dev):
    X = ops.colmajor_empty(D.shape[0], D.shape[1], D.dtype, dev)
    X.copy_(D)
    return X


# ------------------------------------------------------------------ LU
def gbtrf(A, pivots: Pivots, opts=None) -> int:
    """Band LU with partial pivoting (pivots: global 0-based rows).  The
    upper bandwidth of A becomes kl + ku (fill-in), as in SLATE."""
    _need_band(A, "gbtrf")
    if A.op() != Op.NoTrans:
        raise SlateError("gbtrf: pass the band matrix itself")
    with trace_block("gbtrf"):
        kl, ku = _bands(A)
        band_mask(A, kl, ku)
        s, slot, buf = _slab(A)
        if s.KU < tiles_for(kl + ku, s.band_nb):
            raise SlateError("gbtrf: storage has no room for the fill-in (construct with the final kl, ku)")
        comm, Q, me = s.comm, s.Q, s.rank
        m, n, nb, dt, dev = s.m, s.n, s.band_nb, s.dtype, buf.device
        mn = min(m, n)
        kt = -(-mn // nb)
        ipiv = torch.zeros(max(mn, 1), dtype=torch.int64, device=dev)
        infos = torch.zeros(max(kt, 1), dtype=torch.int64, device=dev)
        from .lu import _Pack
        for k in range(kt):
            r0 = k * nb
            kb = min(nb, mn - r0)
            rend = min(m, r0 + kb + kl)
            nr = rend - r0
            owner = k % Q
            pk = _Pack([("P", nr, kb, dt), ("piv", kb, 1, torch.int64)], dev)
            P, pv = pk.get("P"), pk.get("piv")
            with trace_block("gbtrf::panel"):
                if me == owner:
                    Pv = _col_block(s, buf, k, r0, rend)[:, :kb]
                    ops.getrf(Pv, ipiv[r0:r0 + kb], infos[k:k + 1])
                    P.copy_(Pv)
                    pv[:, 0].copy_(ipiv[r0:r0 + kb])
                if Q > 1:
                    comm.bcast(pk.raw, owner)
                    if me != owner:
                        ipiv[r0:r0 + kb].copy_(pv[:, 0])
            with trace_block("gbtrf::update"):
                jhi = (r0 + kb - 1 + ku + kl) // nb
                for j in s.my_cols(k + 1, jhi):
                    C = _col_block(s, buf, j, r0, rend)
                    ops.laswp(C, pv[:, 0], 0, kb)
                    ops.trsm('L', 'L', 'N', 'U', 1.0, P[:kb], C[:kb])
                    if nr > kb:
                        ops.gemm(-1.0, P[kb:], C[:kb], 1.0, C[kb:])
        # the fill-in tiles now hold U: make them part of the matrix
        for j in s.my_cols():
            lo, hi = s.window(j)
            for i in range(lo, hi + 1):
                if not s.tileExists(i, j, slot):
                    s.tileInsert(i, j, slot, data=_col_block(s, buf, j, s.row_offsets[i], s.row_offsets[i + 1])[:, :s.tileNb(j)])
        s.mark_local_modified(slot)
        A.setUpperBandwidth(kl + ku)
        glob = ipiv.cpu().clone()              # panel-relative -> global: host pass
        for k in range(kt):
            r0 = k * nb
            glob[r0:r0 + min(nb, mn - r0)] += r0
        pivots.set(glob[:mn].to(ipiv.device), nb)
        iv = infos[:kt].cpu().tolist()
        info = next((k * nb + v for k, v in enumerate(iv) if v > 0), 0)
        if comm.size > 1:
            big = 1 << 62
            info = int(comm.allreduce_scalar(info if info > 0 else big, "min", torch.int64))
            info = 0 if info >= big else info
        return info


class _DistX:
    """A right-hand side kept 1-D row-cyclic over the band's ranks (tile row
    i on rank i % Q, the owner of band tile column i): the triangular sweeps
    move only the rows of each step's window -- gathered point-to-point onto
    the column's owner, solved / updated there, scattered back -- so no rank
    ever holds the n x nrhs right-hand side (the former solves replicated
    it, docs/INVENTORY.md).  Per-rank workspace: the local rows plus one
    window of (kb + bandwidth) rows."""

    def __init__(self, B, s, dev):
        from ..parallel.redist import redistribute_pieces
        self.s, self.dev = s, dev
        self.dt = s.dtype
        self.m, self.w = B.m(), B.n()
        self.M = _row_cyclic(self.m, self.w, s, self.dt, dev)
        redistribute_pieces(B, self.M)
        self.X = self.M.local_block().data
        self.peak = 0

    def segs(self, lo, hi):
        nb, Q = self.s.band_nb, self.s.Q
        for t in range(lo // nb, -(-hi // nb)):
            a, b = max(lo, t * nb), min(hi, (t + 1) * nb)
            if b > a:
                yield t % Q, a, b, _lrow(self.s, t) + a - t * nb

    def gather(self, lo, hi, root):
        """rows [lo, hi) on ``root`` (None elsewhere)"""
        me = self.s.rank
        W = ops.colmajor_empty(hi - lo, self.w, self.dt, self.dev) if me == root else None
        sends, shapes, dest = {}, {}, {}
        for r, a, b, l in self.segs(lo, hi):
            if r == root:
                if me == root:
                    W[a - lo:b - lo].copy_(self.X[l:l + b - a])
            elif me == r:
                sends.setdefault(root, []).append(self.X[l:l + b - a])
            elif me == root:
                shapes.setdefault(r, []).append((b - a, self.w))
                dest.setdefault(r, []).append(a - lo)
        got = _exchange_pieces(self.s, sends, shapes, self.dt, self.dev)
        for r, lst in got.items():
            for t, o in zip(lst, dest[r]):
                W[o:o + t.shape[0]].copy_(t)
        if W is not None:
            self.peak = max(self.peak, W.numel())
        return W

    def scatter(self, W, lo, hi, root):
        me = self.s.rank
        sends, shapes, dest = {}, {}, {}
        for r, a, b, l in self.segs(lo, hi):
            if r == root:
                if me == root:
                    self.X[l:l + b - a].copy_(W[a - lo:b - lo])
            elif me == root:
                sends.setdefault(r, []).append(W[a - lo:b - lo])
            elif me == r:
                shapes.setdefault(root, []).append((b - a, self.w))
                dest.setdefault(root, []).append(l)
        got = _exchange_pieces(self.s, sends, shapes, self.dt, self.dev)
        for r, lst in got.items():
            for t, l in zip(lst, dest[r]):
                self.X[l:l + t.shape[0]].copy_(t)

    def store(self, B):
        from ..parallel.redist import redistribute_pieces
        self.M.storage.mark_local_modified(self.M.storage.origin_slot)
        redistribute_pieces(self.M, B)


# per-rank peak window (elements) of the last band solve (tests)
BAND_SOLVE_STATS = {"window_elems": 0, "local_elems": 0}


def _note(Xd):
    BAND_SOLVE_STATS["window_elems"] = max(BAND_SOLVE_STATS["window_elems"], Xd.peak)
    BAND_SOLVE_STATS["local_elems"] = max(BAND_SOLVE_STATS["local_elems"], Xd.X.numel())


def _lower_fwd(s, buf, Xd, kd, unit, gpiv=None):
    """X := L^{-1} X (L lower band, bandwidth kd, in the slabs; with gbtrf
    pivots applied step by step when gpiv is given).  Right-looking: the
    window [r0, r0 + kb + kd) goes to the owner of column k and back."""
    n, nb, Q, me = s.n, s.band_nb, s.Q, s.rank
    diag = 'U' if unit else 'N'
    for k in range(-(-min(s.m, n) // nb)):
        r0 = k * nb
        kb = min(nb, n - r0)
        rend = min(n, r0 + kb + kd)
        owner = k % Q
        W = Xd.gather(r0, rend, owner)
        if me == owner:
            if gpiv is not None:
                ops.laswp(W, gpiv[r0:r0 + kb], 0, kb, ioff=r0)
            Pk = _col_block(s, buf, k, r0, rend)[:, :kb]
            ops.trsm('L', 'L', 'N', diag, 1.0, Pk[:kb], W[:kb])
            if rend > r0 + kb:
                ops.gemm(-1.0, Pk[kb:], W[:kb], 1.0, W[kb:])
        Xd.scatter(W, r0, rend, owner)
    _note(Xd)


def _lower_bwd_op(s, buf, Xd, kd, unit, opch):
    """X := op(L)^{-1} X, op = T or C: left-looking, last tile first."""
    n, nb, Q, me = s.n, s.band_nb, s.Q, s.rank
    diag = 'U' if unit else 'N'
    for k in range(-(-n // nb) - 1, -1, -1):
        r0 = k * nb
        kb = min(nb, n - r0)
        rend = min(n, r0 + kb + kd)
        owner = k % Q
        W = Xd.gather(r0, rend, owner)
        if me == owner:
            Pk = _col_block(s, buf, k, r0, rend)[:, :kb]
            if rend > r0 + kb:
                ops.gemm(-1.0, Pk[kb:], W[kb:], 1.0, W[:kb], transA=opch)
            ops.trsm('L', 'L', opch, diag, 1.0, Pk[:kb], W[:kb])
        Xd.scatter(W[:kb] if W is not None else None, r0, r0 + kb, owner)
    _note(Xd)


def _upper_bwd(s, buf, Xd, ku, unit):
    """X := U^{-1} X (U upper band, bandwidth ku): right-looking, last tile first."""
    n, nb, Q, me = s.n, s.band_nb, s.Q, s.rank
    diag = 'U' if unit else 'N'
    for k in range(-(-n // nb) - 1, -1, -1):
        r0 = k * nb
        kb = min(nb, n - r0)
        top = max(0, r0 - ku)
        owner = k % Q
        W = Xd.gather(top, r0 + kb, owner)
        if me == owner:
            Uk = _col_block(s, buf, k, top, r0 + kb)[:, :kb]
            ops.trsm('L', 'U', 'N', diag, 1.0, Uk[r0 - top:], W[r0 - top:])
            if r0 > top:
                ops.gemm(-1.0, Uk[:r0 - top], W[r0 - top:], 1.0, W[:r0 - top])
        Xd.scatter(W, top, r0 + kb, owner)
    _note(Xd)


def _upper_fwd_op(s, buf, Xd, ku, unit, opch):
    """X := op(U)^{-1} X, op = T or C: left-looking, first tile first."""
    n, nb, Q, me = s.n, s.band_nb, s.Q, s.rank
    diag = 'U' if unit else 'N'
    for k in range(-(-n // nb)):
        r0 = k * nb
        kb = min(nb, n - r0)
        top = max(0, r0 - ku)
        owner = k % Q
        W = Xd.gather(top, r0 + kb, owner)
        if me == owner:
            Uk = _col_block(s, buf, k, top, r0 + kb)[:, :kb]
            if r0 > top:
                ops.gemm(-1.0, Uk[:r0 - top], W[:r0 - top], 1.0, W[r0 - top:], transA=opch)
            ops.trsm('L', 'U', opch, diag, 1.0, Uk[r0 - top:], W[r0 - top:])
        Xd.scatter(W[r0 - top:] if W is not None else None, r0, r0 + kb, owner)
    _note(Xd)


def gbtrs(A, pivots, B, opts=None):
    """Solve A X = B with the gbtrf factors (B overwritten)."""
    _need_band(A, "gbtrs")
    with trace_block("gbtrs"):
        s, slot, buf = _slab(A)
        kl, kuf = _bands(A)                 # after gbtrf: ku = kl + ku (fill)
        BAND_SOLVE_STATS.update(window_elems=0, local_elems=0)
        Xd = _DistX(B, s, buf.device)
        _lower_fwd(s, buf, Xd, kl, True, pivots.device(buf.device))
        _upper_bwd(s, buf, Xd, kuf, False)
        Xd.store(B)
        return 0


def gbsv(A, pivots, B, opts=None) -> int:
    info = gbtrf(A, pivots, opts)
    if info == 0:
        gbtrs(A, pivots, B, opts)
    return info


# ------------------------------------------------------------------ Cholesky
def _band_conj_transpose(src, dst):
    """dst := src^H for square band storages with mirrored windows (tile
    (i, j) of dst = tile (j, i) of src, conjugate-transposed).  The slabs
    (O(n bandwidth) words) are exchanged by ONE all-gather."""
    ss, sd = src.storage, dst.storage
    sslot, buf = ss.band_slot(), None
    buf = ss.sync_slab(sslot)
    dslot = sd.band_slot()
    dbuf = sd.get_slab(dslot)
    comm = ss.comm
    rows, ml = buf.shape[0], max(1, max(ss.nloc, 1))
    from ..core.storage import numroc
    mx = max(1, max(numroc(ss.n, ss.band_nb, r, ss.Q) for r in range(ss.Q)))
    pad = torch.zeros((mx, rows), dtype=ss.dtype, device=buf.device)
    if ss.nloc:
        pad[:ss.nloc].copy_(buf[:, :ss.nloc].mT)
    allp = comm.allgather(pad) if comm.size > 1 else pad.unsqueeze(0)
    for j in sd.my_cols():
        lo, hi = sd.window(j)
        for i in range(lo, hi + 1):
            # source tile (j, i): column i of src, owned by rank i % Q
            r = ss.slab_row(ss.row_offsets[j], i)
            c = (i // ss.Q) * ss.band_nb
            src_t = allp[i % ss.Q][c:c + ss.tileNb(i), r:r + ss.tileMb(j)]      # (tile (j, i))^T
            dt = _col_block(sd, dbuf, j, sd.row_offsets[i], sd.row_offsets[i + 1])[:, :sd.tileNb(j)]
            tmp = ops.colmajor_empty(dt.shape[0], dt.shape[1], dt.dtype, dt.device)
            tmp.copy_(src_t.conj() if dt.dtype.is_complex else src_t)
            dt.copy_(tmp)
    sd.mark_local_modified(dslot)


def _to_lower_band(A):
    """Lower-stored copy of an Upper-stored Hermitian band matrix."""
    from ..core.matrix import HermitianBandMatrix
    s = A.storage
    L = HermitianBandMatrix(Uplo.Lower, s.n, A.bandwidth(), nb=s.band_nb, comm=s.comm, dtype=s.dtype,
                            device=s.device)
    L.insertLocalTiles(device=s.device.index if s.device.type == "cuda" else -1)
    _band_conj_transpose(A, L)
    return L


def pbtrf(A, opts=None) -> int:
    """Band Cholesky A = L L^H of a Hermitian band matrix (kd = bandwidth)."""
    _need_band(A, "pbtrf")
    with trace_block("pbtrf"):
        if A.uploPhysical() == Uplo.Upper:
            band_mask(A, 0, A.bandwidth())
            L = _to_lower_band(A)
            info = pbtrf(L, opts)
            _band_conj_transpose(L, A)              # A = U = L^H
            A._chol_lower = L
            return info
        kd = A.bandwidth()
        band_mask(A, kd, 0)
        s, slot, buf = _slab(A)
        comm, Q, me = s.comm, s.Q, s.rank
        n, nb, dt, dev = s.n, s.band_nb, s.dtype, buf.device
        ct = conj_trans(dt)
        kt = -(-n // nb)
        infos = torch.zeros(max(kt, 1), dtype=torch.int64, device=dev)
        for k in range(kt):
            r0 = k * nb
            kb = min(nb, n - r0)
            rend = min(n, r0 + kb + kd)
            nr = rend - r0
            owner = k % Q
            P = ops.colmajor_empty(nr, kb, dt, dev)
            with trace_block("pbtrf::panel"):
                if me == owner:
                    Pv = _col_block(s, buf, k, r0, rend)[:, :kb]
                    ops.potrf('L', Pv[:kb], infos[k:k + 1])
                    if nr > kb:
                        ops.trsm('R', 'L', ct, 'N', 1.0, Pv[:kb], Pv[kb:])
                    P.copy_(Pv)
                if Q > 1:
                    comm.bcast(P, owner)
            with trace_block("pbtrf::update"):
                for j in s.my_cols(k + 1, (rend - 1) // nb):
                    off = s.col_offsets[j] - r0
                    w = min(s.tileNb(j), nr - off)
                    if w <= 0:
                        continue
                    Pj = P[off:nr]
                    C = _col_block(s, buf, j, s.col_offsets[j], rend)[:, :w]
                    ops.gemm(-1.0, Pj, Pj[:w], 1.0, C, 'N', ct, _LOWER_MASK)
        s.mark_local_modified(slot)
        iv = infos[:kt].cpu().tolist()
        info = next((k * nb + v for k, v in enumerate(iv) if v > 0), 0)
        if comm.size > 1:
            big = 1 << 62
            info = int(comm.allreduce_scalar(info if info > 0 else big, "min", torch.int64))
            info = 0 if info >= big else info
        return info


def pbtrs(A, B, opts=None):
    """Solve A X = B with the pbtrf factor (B overwritten)."""
    _need_band(A, "pbtrs")
    with trace_block("pbtrs"):
        L = getattr(A, "_chol_lower", None) if A.uploPhysical() == Uplo.Upper else A
        if L is None:
            raise SlateError("pbtrs: factor with pbtrf first")
        s, slot, buf = _slab(L)
        kd = L.bandwidth()
        BAND_SOLVE_STATS.update(window_elems=0, local_elems=0)
        Xd = _DistX(B, s, buf.device)
        _lower_fwd(s, buf, Xd, kd, False)
        _lower_bwd_op(s, buf, Xd, kd, False, conj_trans(s.dtype))
        Xd.store(B)
        return 0


def pbsv(A, B, opts=None) -> int:
    info = pbtrf(A, opts)
    if info == 0:
        pbtrs(A, B, opts)
    return info


# ------------------------------------------------------------------ tbsm
def tbsm(side, alpha, A, B, pivots=None, opts=None):
    """op(A) X = alpha B (Left) or X op(A) = alpha B (Right) with A a
    triangular band matrix; with ``pivots`` (gbtrf's, A its unit lower
    factor) the row interchanges are applied step by step (tbsmPivots)."""
    _need_band(A, "tbsm")
    with trace_block("tbsm"):
        side = Side(side) if not isinstance(side, Side) else side
        s, slot, buf = _slab(A)
        up = A.uploPhysical()
        opA = A.op()
        unit = getattr(A, "_diag", Diag.NonUnit) == Diag.Unit
        kd = A._kl if up == Uplo.Lower else A._ku
        BAND_SOLVE_STATS.update(window_elems=0, local_elems=0)
        if side == Side.Right:
            # X op(A) = alpha B  <=>  op(A)^T X^T = alpha B^T: B^T goes to the
            # row-cyclic layout by one transposing redistribution
            from .blas3 import _copy_out
            opT = {Op.NoTrans: 'T', Op.Trans: 'N', Op.ConjTrans: 'N'}[opA]
            conj = opA == Op.ConjTrans
            Xd = _DistX(B.conj_transpose() if conj else B.transpose(), s, buf.device)
            _tri_dispatch(s, buf, Xd, up, opT, kd, unit, None)
            if alpha != 1.0 and Xd.X.numel():
                ops.gescale(complex(alpha).conjugate() if conj else alpha, Xd.X)
            Xd.M.storage.mark_local_modified(Xd.M.storage.origin_slot)
            _copy_out(Xd.M.conj_transpose() if conj else Xd.M.transpose(), B)
            return 0
        Xd = _DistX(B, s, buf.device)
        if alpha != 1.0 and Xd.X.numel():
            ops.gescale(alpha, Xd.X)
        opch = {Op.NoTrans: 'N', Op.Trans: 'T', Op.ConjTrans: 'C'}[opA]
        _tri_dispatch(s, buf, Xd, up, opch, kd, unit, pivots.device(buf.device) if pivots is not None else None)
        Xd.store(B)
        return 0


def _tri_dispatch(s, buf, Xd, up, opch, kd, unit, gpiv):
    if up == Uplo.Lower and opch == 'N':
        _lower_fwd(s, buf, Xd, kd, unit, gpiv)
    elif up == Uplo.Lower:
        _lower_bwd_op(s, buf, Xd, kd, unit, opch)
    elif opch == 'N':
        _upper_bwd(s, buf, Xd, kd, unit)
    else:
        _upper_fwd_op(s, buf, Xd, kd, unit, opch)


# ------------------------------------------------------------------ BLAS-3
_CHUNK = 512


def _stored_rows(s, j):
    lo, hi = s.window(j)
    return s.row_offsets[lo], s.row_offsets[hi + 1]


def _row_cyclic(rows, cols, s, dt, dev):
    """A rows x cols matrix 1-D row-cyclic over the band's ranks with the
    band tile size: tile row i lives on rank i % Q at local rows
    (i // Q) nb -- the rows of B / C that meet band tile column i."""
    from ..core.matrix import Matrix
    M = Matrix(rows, cols, nb=max(1, cols), mb=s.band_nb, p=s.Q, q=1, comm=s.comm, dtype=dt, device=dev)
    M.insertLocalTiles(device=dev if dev.type == "cuda" else -1)
    return M


def _lrow(s, i):
    return (i // s.Q) * s.band_nb


def _exchange_pieces(s, sends, recv_shapes, dt, dev):
    """sends {peer: [tensor, ...]}, recv_shapes {peer: [(r, c), ...]}, both
    in an order every rank derives from the same global enumeration: one
    batched send/recv per peer (flattened), returns {peer: [tensor, ...]}."""
    sb, rb = {}, {}
    for r, ts in sends.items():
        sb[r] = torch.cat([t.t().contiguous().reshape(-1) for t in ts]) if ts else None
    for r, shp in recv_shapes.items():
        rb[r] = torch.empty(sum(a * b for a, b in shp), dtype=dt, device=dev)
    sb = {r: t for r, t in sb.items() if t is not None and t.numel()}
    rb = {r: t for r, t in rb.items() if t.numel()}
    if sb or rb:
        s.comm.exchange(sb, rb)
    out = {}
    for r, shp in recv_shapes.items():
        buf, o, lst = rb.get(r), 0, []
        for (a, b) in shp:
            lst.append(buf[o:o + a * b].reshape(b, a).t() if a * b else torch.empty(a, b, dtype=dt, device=dev))
            o += a * b
        out[r] = lst
    return out


def _band_product(s, buf, Bl, Cl, w, mode, up=None):
    """Cl (this rank's row-cyclic part of C, w columns) += the band product
    with Bl (row-cyclic part of B):
      mode 'N': C += A B -- each local column j gives a partial block for
                the tile rows of its window, routed to their owners;
      mode 'T'/'C': C += op(A) B -- column j needs the B tiles of its
                window (fetched from their owners), produces tile row j;
      mode 'H': A Hermitian stored in triangle ``up``: the stored part as
                'N' and its conjugate transpose (diagonal tile counted
                once) as 'C'.
    Every transfer is point-to-point between the owners; nothing is
    replicated or all-reduced."""
    dt, dev = buf.dtype, buf.device
    me, Q = s.rank, s.Q
    ct = conj_trans(dt)
    cols = list(range(s.nt))

    def tile_rows(i):
        return s.row_offsets[i], s.row_offsets[i + 1]

    do_n = mode in ('N', 'H')
    do_t = mode in ('T', 'C', 'H')
    tch = ct if mode in ('C', 'H') else 'T'
    # ---- 'N' part: pieces (i, j) from owner(j) to owner(i)
    if do_n:
        sends, shapes, mine = {}, {}, []
        for j in cols:
            lo, hi = s.window(j)
            oj = j % Q
            for i in range(lo, hi + 1):
                oi = i % Q
                if oj == me and oi != me:
                    sends.setdefault(oi, []).append((i, j))
                elif oi == me and oj != me:
                    shapes.setdefault(oj, []).append((i, j))
                elif oi == me and oj == me:
                    mine.append((i, j))
        parts = {}
        for j in s.my_cols():
            g0, g1 = _stored_rows(s, j)
            S = _col_block(s, buf, j, g0, g1)
            cj0, cj1 = s.col_offsets[j], s.col_offsets[j + 1]
            if mode == 'H' and dt.is_complex:
                # the diagonal of a Hermitian matrix is real (its stored
                # imaginary part is ignored, as in hemm)
                S2 = ops.colmajor_empty(S.shape[0], S.shape[1], dt, dev)
                S2.copy_(S)
                d0 = cj0 - g0
                torch.diagonal(S2[d0:d0 + (cj1 - cj0)]).imag.zero_()
                S = S2
            P = ops.colmajor_zeros(g1 - g0, w, dt, dev)
            if w:
                ops.gemm(1.0, S, Bl[_lrow(s, j):_lrow(s, j) + (cj1 - cj0)], 0.0, P)
            parts[j] = (g0, P)

        def piece(i, j):
            g0, P = parts[j]
            r0, r1 = tile_rows(i)
            return P[r0 - g0:r1 - g0]
        snd = {r: [piece(i, j) for (i, j) in lst] for r, lst in sends.items()}
        rsh = {r: [(tile_rows(i)[1] - tile_rows(i)[0], w) for (i, j) in lst] for r, lst in shapes.items()}
        got = _exchange_pieces(s, snd, rsh, dt, dev)
        for (i, j) in mine:
            r0, r1 = tile_rows(i)
            ops.geadd(1.0, piece(i, j), 1.0, Cl[_lrow(s, i):_lrow(s, i) + (r1 - r0)])
        for r, lst in shapes.items():
            for (i, j), T in zip(lst, got[r]):
                r0, r1 = tile_rows(i)
                ops.geadd(1.0, T, 1.0, Cl[_lrow(s, i):_lrow(s, i) + (r1 - r0)])
    # ---- 'T' part: B tiles (i) of column j's window from owner(i) to owner(j)
    if do_t:
        sends, shapes = {}, {}
        for j in cols:
            lo, hi = s.window(j)
            oj = j % Q
            for i in range(lo, hi + 1):
                oi = i % Q
                if oi == me and oj != me:
                    sends.setdefault(oj, []).append((i, j))
                elif oj == me and oi != me:
                    shapes.setdefault(oi, []).append((i, j))
        snd = {r: [Bl[_lrow(s, i):_lrow(s, i) + (tile_rows(i)[1] - tile_rows(i)[0])] for (i, j) in lst]
               for r, lst in sends.items()}
        rsh = {r: [(tile_rows(i)[1] - tile_rows(i)[0], w) for (i, j) in lst] for r, lst in shapes.items()}
        got = _exchange_pieces(s, snd, rsh, dt, dev)
        halo = {}
        for r, lst in shapes.items():
            for (i, j), T in zip(lst, got[r]):
                halo[(i, j)] = T
        for j in s.my_cols():
            g0, g1 = _stored_rows(s, j)
            lo, hi = s.window(j)
            S = _col_block(s, buf, j, g0, g1)
            cj0, cj1 = s.col_offsets[j], s.col_offsets[j + 1]
            Bh = ops.colmajor_empty(g1 - g0, w, dt, dev)
            for i in range(lo, hi + 1):
                r0, r1 = tile_rows(i)
                src = Bl[_lrow(s, i):_lrow(s, i) + (r1 - r0)] if i % Q == me else halo[(i, j)]
                Bh[r0 - g0:r1 - g0].copy_(src)
            Sx = S
            if mode == 'H':
                Sx = ops.colmajor_empty(S.shape[0], S.shape[1], dt, dev)
                Sx.copy_(S)
                d0 = cj0 - g0
                ops.geset(0.0, 0.0, Sx[d0:d0 + (cj1 - cj0)], uplo='U' if up == Uplo.Lower else 'L')
            if w:
                ops.gemm(1.0, Sx, Bh, 1.0, Cl[_lrow(s, j):_lrow(s, j) + (cj1 - cj0)], transA=tch)


def _band_mm(alpha, s, buf, B, beta, C, mode, up=None):
    """C = alpha op(A) B + beta C for the band A in slabs ``buf`` (Left)."""
    from ..parallel.redist import redistribute_pieces
    dt, dev = buf.dtype, buf.device
    w = B.n()
    Bw = _row_cyclic(B.m(), w, s, dt, dev)
    redistribute_pieces(B, Bw)
    Cw = _row_cyclic(C.m(), w, s, dt, dev)
    lbB, lbC = Bw.local_block(), Cw.local_block()
    Cl = lbC.data[:lbC.mloc, :lbC.nloc]
    Cl.zero_()
    _band_product(s, buf, lbB.data[:lbB.mloc, :lbB.nloc], Cl, w, mode, up)
    if beta != 0:
        Ct = _row_cyclic(C.m(), w, s, dt, dev)
        redistribute_pieces(C, Ct)
        lt = Ct.local_block()
        if lt.mloc and lt.nloc:
            ops.geadd(alpha, Cl, beta, lt.data[:lt.mloc, :lt.nloc])
        Ct.storage.mark_local_modified(Ct.storage.origin_slot)
        redistribute_pieces(Ct, C)
    else:
        if alpha != 1 and lbC.mloc and lbC.nloc:
            ops.gescale(alpha, Cl)
        Cw.storage.mark_local_modified(Cw.storage.origin_slot)
        redistribute_pieces(Cw, C)
    return C


def gbmm(alpha, A, B, beta, C, opts=None):
    """C = alpha op(A) B + beta C with A a band matrix (op from A's view):
    B and C in 1-D row-cyclic work layouts matched to the band's column
    ownership, point-to-point pieces between owners (_band_product)."""
    _need_band(A, "gbmm")
    with trace_block("gbmm"):
        band_mask(A, A._kl, A._ku)
        s, slot, buf = _slab(A)
        opA = A.op()
        mode = {Op.NoTrans: 'N', Op.Trans: 'T', Op.ConjTrans: 'C'}[opA]
        return _band_mm(alpha, s, buf, B, beta, C, mode)


def hbmm(side, alpha, A, B, beta, C, opts=None):
    """C = alpha A B + beta C (Left) or alpha B A + beta C (Right), A a
    Hermitian band matrix: the stored triangle is read twice (as is and
    conjugate-transposed, diagonal once), no replication of B."""
    _need_band(A, "hbmm")
    with trace_block("hbmm"):
        side = Side(side) if not isinstance(side, Side) else side
        kd = A.bandwidth()
        up = A.uploPhysical()
        band_mask(A, kd, 0) if up == Uplo.Lower else band_mask(A, 0, kd)
        s, slot, buf = _slab(A)
        if side == Side.Left:
            return _band_mm(alpha, s, buf, B, beta, C, 'H', up)
        # Right: C^H = A B^H + ... (A Hermitian)
        cplx = s.dtype.is_complex
        tr = (lambda X: X.conj_transpose()) if cplx else (lambda X: X.transpose())
        cj = (lambda v: complex(v).conjugate()) if cplx else (lambda v: v)
        return _band_mm(cj(alpha), s, buf, tr(B), cj(beta), tr(C), 'H', up) and C
