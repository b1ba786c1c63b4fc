"""Piece-level redistribution between two distributed matrices.

The reference moves whole tiles with blocking send/recv pairs, one tile at
a time (`src/redistribute.cc:20-150`), and gathers to one rank for the band
and print paths (`include/slate/Matrix.hh:775-822`).  Here one call moves an
arbitrary logical matrix ``op(A)`` into ``op(B)``:

* the logical index space is cut at the union of A's and B's tile
  boundaries (mapped through each view's op), so every *piece* has exactly
  one source rank and one destination rank -- tile sizes, offsets, grids,
  transposes and conjugations may all differ between A and B;
* the pieces a rank sends to one peer are packed into ONE contiguous
  message (packing applies op(A), unpacking applies op(B), both with the
  gecopy kernel, which also converts precision), and all messages of the
  call go out as one batched point-to-point exchange (an RCCL group over
  xGMI: every peer pair uses its own link concurrently);
* ``uplo`` restricts the copy to one logical triangle (Hermitian /
  triangular storage): pieces outside it are never sent, pieces crossing
  it are masked at the destination, so the other triangle of B is never
  touched (LAPACK semantics).

Nothing is gathered: each rank sends and receives only the elements whose
owner changes.  Host planning is O(#pieces) per call.
"""
from __future__ import annotations

import bisect

import torch

from .. import ops
from ..core.enums import Op, Uplo


def _logical_bounds(X, along_rows: bool):
    """Cut points (0 .. len) of op(X)'s logical rows (or cols) at X's tile
    boundaries."""
    s = X.storage
    R0, C0 = X.global_offsets()
    um, un = X._um(), X._un()
    # logical rows of op(X) are stored rows (NoTrans) or stored cols (Trans)
    use_rows = along_rows == (X.op() == Op.NoTrans)
    offs, base, length = (s.row_offsets, R0, um) if use_rows else (s.col_offsets, C0, un)
    lo = bisect.bisect_right(offs, base)
    hi = bisect.bisect_left(offs, base + length)
    cuts = [0] + [o - base for o in offs[lo:hi]] + [length]
    return sorted(set(cuts)), use_rows


def _stored_tile(X, lr, lc):
    """Stored tile (gi, gj) and in-tile offsets of logical element (lr, lc) of op(X)."""
    s = X.storage
    R0, C0 = X.global_offsets()
    if X.op() == Op.NoTrans:
        gr, gc = R0 + lr, C0 + lc
    else:
        gr, gc = R0 + lc, C0 + lr
    gi = bisect.bisect_right(s.row_offsets, gr) - 1
    gj = bisect.bisect_right(s.col_offsets, gc) - 1
    return gi, gj, gr - s.row_offsets[gi], gc - s.col_offsets[gj]


def _op_code(X):
    return {Op.NoTrans: 'N', Op.Trans: 'T', Op.ConjTrans: 'C'}[X.op()]


def _stored_piece(X, slot, lr0, lr1, lc0, lc1, create=False):
    """Local tensor (stored orientation) of the logical piece [lr0,lr1)x[lc0,lc1)."""
    s = X.storage
    gi, gj, oi, oj = _stored_tile(X, lr0, lc0)
    h, w = lr1 - lr0, lc1 - lc0
    sh, sw = (h, w) if X.op() == Op.NoTrans else (w, h)
    t = s.tile_data(gi, gj, slot)
    if t is None:
        if not create:
            raise RuntimeError(f"redistribute: local tile ({gi},{gj}) has no instance")
        t = s.tileInsert(gi, gj, slot)
    return t[oi:oi + sh, oj:oj + sw]


def _classify(uplo, r0, r1, c0, c1):
    """'all', 'none' or 'diag' for a logical piece against a triangle."""
    if uplo is None or uplo == Uplo.General:
        return 'all'
    if uplo == Uplo.Lower:
        if r1 - 1 < c0:
            return 'none'
        if r0 >= c1 - 1:
            return 'all'
    else:
        if r0 > c1 - 1:
            return 'none'
        if r1 - 1 <= c0:
            return 'all'
    return 'diag'


def _slot_of(X):
    s = X.storage
    if s.origin_slot is not None:
        return s.origin_slot
    from ..core.storage import DEV, HOST
    return DEV if s.device.type == "cuda" else HOST


def _ready(X, slot):
    s = X.storage
    if s.bc is not None and s.local:
        s.prepare_local(slot)
    elif s.bc is None:
        s.sync_origin()


def redistribute_pieces(A, B, uplo=None):
    """B := op(A) for any two distributed views of the same logical shape.

    uplo (logical, of op(B)): copy only that triangle; B's other elements
    are left untouched.  Collective over A's communicator."""
    m, n = A.m(), A.n()
    if (m, n) != (B.m(), B.n()):
        raise ValueError(f"redistribute: shape mismatch {m}x{n} vs {B.m()}x{B.n()}")
    if m == 0 or n == 0:
        return B
    sA, sB = A.storage, B.storage
    comm = sA.comm
    me = comm.rank
    slotA, slotB = _slot_of(A), _slot_of(B)
    _ready(A, slotA)
    if sB.bc is not None:
        if slotB not in sB.local:
            B.insertLocalTiles(device=sB.device if slotB == 1 else -1)
        _ready(B, slotB)
    rows = sorted(set(_logical_bounds(A, True)[0]) | set(_logical_bounds(B, True)[0]))
    cols = sorted(set(_logical_bounds(A, False)[0]) | set(_logical_bounds(B, False)[0]))
    opA, opB = _op_code(A), _op_code(B)
    dtA, dtB = sA.dtype, sB.dtype
    devA = sA.device_of(slotA)
    devB = sB.device_of(slotB)
    # plan: pieces per (src, dst) pair, in a deterministic order on all ranks
    send_plan, recv_plan, local = {}, {}, []
    for ri in range(len(rows) - 1):
        r0, r1 = rows[ri], rows[ri + 1]
        for ci in range(len(cols) - 1):
            c0, c1 = cols[ci], cols[ci + 1]
            kind = _classify(uplo, r0, r1, c0, c1)
            if kind == 'none':
                continue
            ga = _stored_tile(A, r0, c0)
            gb = _stored_tile(B, r0, c0)
            src = sA.tileRank((ga[0], ga[1]))
            dst = sB.tileRank((gb[0], gb[1]))
            if src != me and dst != me:
                continue
            pc = (r0, r1, c0, c1, kind)
            if src == me and dst == me:
                local.append(pc)
            elif src == me:
                send_plan.setdefault(dst, []).append(pc)
            else:
                recv_plan.setdefault(src, []).append(pc)
    # pack: logical orientation, column-major per piece
    sends = {}
    for dst, pcs in send_plan.items():
        tot = sum((p[1] - p[0]) * (p[3] - p[2]) for p in pcs)
        buf = torch.empty(tot, dtype=dtA, device=devA)
        off = 0
        for (r0, r1, c0, c1, _) in pcs:
            h, w = r1 - r0, c1 - c0
            ops.gecopy(_stored_piece(A, slotA, r0, r1, c0, c1), buf[off:off + h * w].view(w, h).t(),
                       trans=opA)
            off += h * w
        sends[dst] = buf
    recvs = {}
    for src, pcs in recv_plan.items():
        tot = sum((p[1] - p[0]) * (p[3] - p[2]) for p in pcs)
        recvs[src] = torch.empty(tot, dtype=dtA, device=devA)
    # local pieces are read before the exchange lands anything (A and B may
    # alias, e.g. an in-place transpose of a square matrix's own storage)
    staged = []
    for (r0, r1, c0, c1, kind) in local:
        h, w = r1 - r0, c1 - c0
        L = ops.colmajor_empty(h, w, dtA, devA)
        ops.gecopy(_stored_piece(A, slotA, r0, r1, c0, c1), L, trans=opA)
        staged.append(((r0, r1, c0, c1, kind), L))
    comm.exchange(sends, recvs)
    for pc, L in staged:
        _unpack(B, slotB, pc, L, uplo, opB, devB)
    for src, pcs in recv_plan.items():
        buf = recvs[src]
        off = 0
        for pc in pcs:
            r0, r1, c0, c1, _ = pc
            h, w = r1 - r0, c1 - c0
            _unpack(B, slotB, pc, buf[off:off + h * w].view(w, h).t(), uplo, opB, devB)
            off += h * w
    sB.mark_local_modified(slotB) if sB.bc is not None else None
    if sB.bc is None:
        for (r0, r1, c0, c1, _) in local + [p for v in recv_plan.values() for p in v]:
            gi, gj, _, _ = _stored_tile(B, r0, c0)
            sB.tileModified(gi, gj, slotB, True)
    return B


def _unpack(B, slotB, pc, L, uplo, opB, devB):
    """Write logical piece L (column-major, h x w) into B's stored piece."""
    r0, r1, c0, c1, kind = pc
    if L.device != devB:
        L = L.to(devB)
    dst = _stored_piece(B, slotB, r0, r1, c0, c1, create=True)
    if kind == 'all':
        ops.gecopy(L, dst, trans=opB)
        return
    # crosses the diagonal: stored triangle in the stored orientation
    lower = uplo == Uplo.Lower
    d = r0 - c0
    if d == 0:
        u = ('L' if lower else 'U') if opB == 'N' else ('U' if lower else 'L')
        ops.gecopy(L, dst, uplo=u, trans=opB)
        return
    # non-aligned diagonal (tilings differ): column strips
    h, w = L.shape
    for c in range(w):
        gc = c0 + c
        if lower:
            a, b = max(0, gc - r0), h
        else:
            a, b = 0, min(h, gc - r0 + 1)
        if a >= b:
            continue
        piece = L[a:b, c:c + 1]
        if opB == 'N':
            ops.gecopy(piece, dst[a:b, c:c + 1])
        else:
            ops.gecopy(piece, dst[c:c + 1, a:b], trans=opB)
