"""Auxiliary distributed routines: copy (with precision conversion), add,
scale, scale_row_col, set, norm, colNorms, gather, redistribute.

Reference: `src/copy.cc`, `src/add.cc`, `src/scale.cc`,
`src/scale_row_col.cc`, `src/set.cc`, `src/set_lambdas.cc`,
`src/norm.cc:45-170`, `src/colNorms.cc`, `src/redistribute.cc:20-150`,
`include/slate/Matrix.hh:775-822` (gather).

For block-cyclic matrices the element-wise ops are ONE kernel over the
rank's local block (uplo handled in global coordinates by masking per local
tile).  Norms: one local-contribution kernel, then a single all-reduce of a
packed vector (NaN-propagating max as SLATE's mpi_max_nan).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .. import ops
from ..core.enums import Norm, NormScope, Op, Uplo
from ..core.exceptions import SlateError
from ..core.storage import DEV, HOST, l2g
from ._util import target_slot


# ------------------------------------------------------------------ helpers
def _diag_kind(A):
    return getattr(A, "_kind", "general")


def _local_uplo_blocks(A, lb):
    """Yield (local tensor block, uplo) pieces of the local block such that
    applying `uplo` element masks per piece reproduces the GLOBAL triangle.
    Off-diagonal local tiles are full or empty; diagonal tiles get uplo."""
    up = A.uploPhysical()
    if up == Uplo.General:
        yield lb.data, 'G'
        return
    mb, nb = lb.mb, lb.nb
    R0, C0 = lb.grow0, lb.gcol0
    # iterate local tile rows/cols
    rt = _tile_ranges(lb.row_off, lb.mloc, mb, lb.p, lb.pr)
    ct = _tile_ranges(lb.col_off, lb.nloc, nb, lb.q, lb.pc)
    for (r0, r1, gr0) in rt:
        for (c0, c1, gc0) in ct:
            # global (view-relative) row/col ranges of this piece
            vr0, vr1 = gr0 - R0, gr0 - R0 + (r1 - r0) - 1
            vc0, vc1 = gc0 - C0, gc0 - C0 + (c1 - c0) - 1
            blk = lb.data[r0 - lb.row_off:r1 - lb.row_off, c0 - lb.col_off:c1 - lb.col_off]
            if up == Uplo.Lower:
                if vr1 < vc0:
                    continue
                if vr0 >= vc1:
                    yield blk, 'G'
                else:
                    yield from _diag_piece(blk, vr0, vc0, 'L')
            else:
                if vr0 > vc1:
                    continue
                if vr1 <= vc0:
                    yield blk, 'G'
                else:
                    yield from _diag_piece(blk, vr0, vc0, 'U')


def _diag_piece(blk, vr0, vc0, u):
    # piece straddles the diagonal; offset d = vr0 - vc0
    d = vr0 - vc0
    if d == 0:
        yield blk, u
        return
    # general case (non-aligned views): fall back to column-by-column
    m, n = blk.shape
    for c in range(n):
        gc = vc0 + c
        if u == 'L':
            r_start = max(0, gc - vr0)
            if r_start < m:
                yield blk[r_start:, c:c + 1], 'G'
        else:
            r_end = min(m, gc - vr0 + 1)
            if r_end > 0:
                yield blk[:r_end, c:c + 1], 'G'


def _tile_ranges(off, nloc, nb, p, pr):
    """Local index ranges [a, b) split at tile boundaries, with global start."""
    out = []
    a = off
    end = off + nloc
    while a < end:
        b = min(end, (a // nb + 1) * nb)
        out.append((a, b, l2g(a, nb, pr, p)))
        a = b
    return out


def run_on_block_cyclic(A, fn, opts, *others):
    """Run a block-cyclic-only driver on a general-storage matrix by copying
    into a block-cyclic twin and back (redistribute)."""
    from ..core.matrix import Matrix
    s = A.storage
    nb = max(s.tileMb(0) if s.mt else 1, 1)
    B = type(A).__new__(type(A))
    B.__dict__.update(A.__dict__)
    twin = Matrix(A.m(), A.n(), nb=nb, comm=s.comm, dtype=s.dtype, device=s.device)
    twin.insertLocalTiles(device=s.device if s.device.type == "cuda" else -1)
    redistribute(A, twin)
    B.__dict__.update(twin.__dict__)
    B._uplo, B._diag = A._uplo, A._diag
    r = fn(B, opts, *others)
    redistribute(twin, A)
    return r


# --------------------------------------------------------------- dense I/O
def allgather_dense(A) -> torch.Tensor:
    """Return the full m x n logical matrix op(A) on every rank (testing)."""
    s = A.storage
    comm = s.comm
    full = _storage_dense(s)
    R0, C0 = A.global_offsets()
    um, un = A._um(), A._un()
    D = full[R0:R0 + um, C0:C0 + un]
    if A.op() == Op.Trans:
        D = D.transpose(0, 1)
    elif A.op() == Op.ConjTrans:
        D = D.transpose(0, 1).conj()
    return D.contiguous()


def _storage_dense(s) -> torch.Tensor:
    comm = s.comm
    dev = s.device if (s.origin_slot == DEV) else torch.device("cpu")
    full = torch.zeros((s.m, s.n), dtype=s.dtype, device=dev)
    if s.bc is not None and s.local:
        s.sync_origin()
        bc = s.bc
        buf = s.local[s.origin_slot][: bc.mloc, : bc.nloc].to(dev)
        maxm = max(1, max((_numroc_r(s.m, bc.mb, r, bc.p) for r in range(bc.p)), default=1))
        maxn = max(1, max((_numroc_r(s.n, bc.nb, c, bc.q) for c in range(bc.q)), default=1))
        pad = torch.zeros((maxm, maxn), dtype=s.dtype, device=dev)
        pad[: bc.mloc, : bc.nloc] = buf
        allp = comm.allgather(pad) if comm.size > 1 else pad.unsqueeze(0)
        for r in range(min(comm.size, bc.p * bc.q)):
            pr, pc = (r % bc.p, r // bc.p) if bc.order.value == 'C' else (r // bc.q, r % bc.q)
            ml, nl = _numroc_r(s.m, bc.mb, pr, bc.p), _numroc_r(s.n, bc.nb, pc, bc.q)
            if ml == 0 or nl == 0:
                continue
            rows = torch.tensor([l2g(i, bc.mb, pr, bc.p) for i in range(ml)], device=dev)
            cols = torch.tensor([l2g(j, bc.nb, pc, bc.q) for j in range(nl)], device=dev)
            full[rows[:, None], cols[None, :]] = allp[r][:ml, :nl]
        return full
    # per-tile storage: owners broadcast their tiles
    inw = getattr(s, "in_window", None)
    for j in range(s.nt):
        for i in range(s.mt):
            if inw is not None and not inw(i, j):
                continue                      # band storage: tile does not exist anywhere
            owner = s.tileRank((i, j))
            r0, c0 = s.row_offsets[i], s.col_offsets[j]
            mb, nb = s.tileMb(i), s.tileNb(j)
            blk = torch.zeros((mb, nb), dtype=s.dtype, device=dev)
            if owner == comm.rank and s.tileExists(i, j):
                o = s.table.origin(i, j)
                if o < 0:
                    o = s.origin_slot if s.origin_slot is not None else HOST
                s.tileUpdateOrigin(i, j)
                d = s.tile_data(i, j, o)
                if d is not None:
                    blk.copy_(d)
            if comm.size > 1:
                comm.bcast(blk, owner)
            full[r0:r0 + mb, c0:c0 + nb] = blk
    return full


def _numroc_r(n, nb, iproc, nprocs):
    from ..core.storage import numroc
    return numroc(n, nb, iproc, nprocs)


def gather(A, root=0):
    """The whole matrix on ``root`` only (Matrix::gather): a piece-level
    redistribution onto a one-process grid owned by rank 0 (other roots
    get it from rank 0 by one broadcast-free send through the same
    engine)."""
    s = A.storage
    if s.comm.size == 1:
        return allgather_dense(A)
    from ..core.matrix import Matrix
    nb = s.bc.nb if s.bc is not None else max(s.tileNb(0) if s.nt else 1, 1)
    R = Matrix(A.m(), A.n(), nb=nb, p=1, q=1, comm=s.comm, dtype=s.dtype, device=s.device)
    R.insertLocalTiles(device=s.device.index if s.device.type == "cuda" else -1)
    redistribute(A, R)
    D = None
    if s.comm.rank == 0:
        lb = R.local_block()
        D = lb.data[:A.m(), :A.n()].clone()
    if root != 0:
        import torch.distributed as dist
        if s.comm.rank in (0, root):
            buf = D if s.comm.rank == 0 else torch.empty((A.n(), A.m()), dtype=s.dtype, device=s.device).t()
            t = buf.t().contiguous() if s.comm.rank == 0 else torch.empty((A.n(), A.m()), dtype=s.dtype,
                                                                            device=s.device)
            if s.comm.rank == 0:
                dist.send(t, s.comm.ranks[root] if hasattr(s.comm, "ranks") else root, group=s.comm.group)
                D = None
            else:
                dist.recv(t, s.comm.ranks[0] if hasattr(s.comm, "ranks") else 0, group=s.comm.group)
                D = t.t()
        else:
            D = None
    return D


def from_dense(A, D: torch.Tensor):
    """Scatter a replicated dense (logical op(A)-shaped) tensor into A."""
    s = A.storage
    if A.op() == Op.Trans:
        D = D.transpose(0, 1)
    elif A.op() == Op.ConjTrans:
        D = D.transpose(0, 1).conj()
    R0, C0 = A.global_offsets()
    if s.bc is not None:
        if not s.local:
            A.insertLocalTiles(device=s.device if s.device.type == "cuda" else -1)
        bc = s.bc
        lb = A.local_block()
        if bc.pr >= 0 and lb.mloc and lb.nloc:
            rows = torch.tensor([l2g(lb.row_off + i, bc.mb, bc.pr, bc.p) - R0 for i in range(lb.mloc)],
                                device=D.device)
            cols = torch.tensor([l2g(lb.col_off + j, bc.nb, bc.pc, bc.q) - C0 for j in range(lb.nloc)],
                                device=D.device)
            lb.data.copy_(D[rows[:, None], cols[None, :]].to(lb.data.device, lb.data.dtype))
        s.mark_local_modified(s.origin_slot)
        return A
    inw = getattr(s, "in_window", None)
    for j in range(A._nt):
        for i in range(A._mt):
            gi, gj = A.ioffset + i, A.joffset + j
            if inw is not None and not inw(gi, gj):
                continue
            if s.tileIsLocal(gi, gj):
                d = s.tile_data(gi, gj, s.origin_slot if s.origin_slot is not None else HOST)
                if d is None:
                    d = s.tileInsert(gi, gj, s.slot_of(s.device) if s.device.type == "cuda" else HOST)
                r0 = s.row_offsets[gi] - R0
                c0 = s.col_offsets[gj] - C0
                d.copy_(D[r0:r0 + d.shape[0], c0:c0 + d.shape[1]])
    return A


# -------------------------------------------------------------- redistribute
def redistribute(A, B, opts=None):
    """B = A for arbitrary distributions / ops (tile-level send/recv,
    `src/redistribute.cc:20-150`); elements outside B's stored triangle are
    ignored for trapezoid types."""
    sA, sB = A.storage, B.storage
    comm = sA.comm
    if A.m() != B.m() or A.n() != B.n():
        raise SlateError("redistribute: dimension mismatch")
    # fast path: identical block-cyclic layouts and ops
    if sA.bc is not None and sB.bc is not None and sA.local and sB.local and A.op() == B.op() and \
            (sA.bc.mb, sA.bc.nb, sA.bc.p, sA.bc.q, sA.bc.order) == (sB.bc.mb, sB.bc.nb, sB.bc.p, sB.bc.q, sB.bc.order) \
            and A.global_offsets() == B.global_offsets():
        la, lbk = A.local_block(), B.local_block()
        ops.gecopy(la.data, lbk.data)
        sB.mark_local_modified(sB.origin_slot)
        return B
    # general path: piece-level batched point-to-point (parallel/redist.py);
    # trapezoid targets receive only their stored triangle
    from ..parallel.redist import redistribute_pieces
    up = B.uplo() if getattr(B, "_kind", "general") != "general" else None
    return redistribute_pieces(A, B, uplo=up)


def copy_conj_transpose(A, B):
    """B = A^H restricted to B's stored triangle (A's matching triangle is
    read; every other element of B is left untouched)."""
    from ..parallel.redist import redistribute_pieces
    up = B.uplo() if B.uploPhysical() != Uplo.General else None
    return redistribute_pieces(A.conj_transpose(), B, uplo=up)


# ------------------------------------------------------------------ element-wise
def _bc_pieces(A, opts=None):
    s = A.storage
    if s.bc is None:
        raise SlateError("element-wise op requires block-cyclic storage")
    slot = target_slot(A, opts) if opts is not None else s.origin_slot
    lb = A.local_block(slot)
    return s, slot, lb


def set(offdiag, diag, A, opts=None):
    """A = offdiag off the diagonal, diag on it (src/set.cc)."""
    s, slot, lb = _bc_pieces(A, opts)
    if lb.mloc and lb.nloc:
        for blk, u in _local_uplo_blocks(A, lb):
            _set_block(blk, offdiag, diag, lb, A, u)
    s.mark_local_modified(slot)
    return A


def _set_block(blk, off, dg, lb, A, u):
    ops.geset(off, off, blk, uplo=u)
    m, n = blk.shape
    if m == 0 or n == 0:
        return
    # the global diagonal crosses a block-cyclic local block in runs (one per
    # diagonal tile it owns): find them and set each run's square
    for (i0, j0, k) in _diag_runs(blk, lb):
        ops.geset(off, dg, blk[i0:i0 + k, j0:j0 + k], uplo=u)


def _diag_runs(blk, lb):
    gr, gc = _piece_globals(blk, lb)
    cpos = {g: j for j, g in enumerate(gc)}
    runs = []
    i = 0
    m = len(gr)
    while i < m:
        j = cpos.get(gr[i])
        if j is None:
            i += 1
            continue
        k = 1
        while i + k < m and j + k < len(gc) and gr[i + k] == gr[i] + k and gc[j + k] == gc[j] + k:
            k += 1
        runs.append((i, j, k))
        i += k
    return runs


def set_diag(A, value, opts=None):
    """A(i, i) = value for the stored diagonal (block-cyclic): one geset per
    run of locally owned diagonal elements."""
    s, slot, lb = _bc_pieces(A, opts)
    if lb.mloc and lb.nloc:
        for (i0, j0, k) in _diag_runs(lb.data, lb):
            blk = lb.data[i0:i0 + k, j0:j0 + k]
            ops.geset(0.0, value, blk, uplo='D')
    s.mark_local_modified(slot)
    return A


def set_diag_imag_zero(A, opts=None):
    """Drop the imaginary part of the stored diagonal (Hermitian operands:
    LAPACK assumes it is zero)."""
    s, slot, lb = _bc_pieces(A, opts)
    if lb.mloc and lb.nloc and s.dtype.is_complex:
        for (i0, j0, k) in _diag_runs(lb.data, lb):
            d = torch.diagonal(lb.data[i0:i0 + k, j0:j0 + k])
            d.imag.zero_()
    s.mark_local_modified(slot)
    return A


def scale(numer, denom, A, opts=None):
    """A = (numer / denom) A (src/scale.cc; overflow-safe ratio like lascl)."""
    s, slot, lb = _bc_pieces(A, opts)
    alpha = numer / denom
    if lb.mloc and lb.nloc:
        for blk, u in _local_uplo_blocks(A, lb):
            ops.gescale(alpha, blk, uplo=u)
    s.mark_local_modified(slot)
    return A


def add(alpha, A, beta, B, opts=None):
    """B = alpha A + beta B (src/add.cc)."""
    sB = B.storage
    if not (A.storage.bc is not None and sB.bc is not None and A.op() == B.op() == Op.NoTrans):
        raise SlateError("add: block-cyclic NoTrans matrices required")
    if not _same_layout(A, B):
        # bring A onto B's layout first (piece-level exchange), then add locally
        T = B.emptyLike()
        T.insertLocalTiles(device=sB.device.index if sB.device.type == "cuda" else -1)
        redistribute(A, T)
        A = T
    la, lb = A.local_block(), B.local_block()
    if lb.mloc and lb.nloc:
        if B.uploPhysical() == Uplo.General:
            ops.geadd(alpha, la.data, beta, lb.data)
        else:
            pa = list(_local_uplo_blocks(A, la))
            pb = list(_local_uplo_blocks(B, lb))
            for (xa, u), (xb, _) in zip(pa, pb):
                ops.geadd(alpha, xa, beta, xb, uplo=u)
    sB.mark_local_modified(sB.origin_slot)
    return B


def _same_layout(A, B):
    """True when op(A) and op(B) put every element on the same rank at the
    same local position (then copies are purely local)."""
    a, b = A.storage.bc, B.storage.bc
    if a is None or b is None or A.op() != B.op():
        return False
    if (a.mb, a.nb, a.p, a.q, a.order, a.pr, a.pc) != (b.mb, b.nb, b.p, b.q, b.order, b.pr, b.pc):
        return False
    if A.storage.comm is not B.storage.comm and A.storage.comm.ranks != B.storage.comm.ranks:
        return False
    return A.global_offsets() == B.global_offsets() and (A.m(), A.n()) == (B.m(), B.n())


def copy(A, B, opts=None):
    """B = A with precision conversion (src/copy.cc): a local copy when the
    layouts coincide, the piece-level redistribution otherwise."""
    if _same_layout(A, B):
        la, lb = A.local_block(), B.local_block()
        if lb.mloc and lb.nloc:
            if B.uploPhysical() == Uplo.General:
                ops.gecopy(la.data, lb.data)
            else:
                # B's stored-triangle pieces; A's data at the same local offsets
                # (identical layouts), whatever A's own structure
                ldb = max(1, lb.data.stride(1))
                for xb, u in _local_uplo_blocks(B, lb):
                    off = xb.storage_offset() - lb.data.storage_offset()
                    r, c = off % ldb, off // ldb
                    ops.gecopy(la.data[r:r + xb.shape[0], c:c + xb.shape[1]], xb, uplo=u)
        B.storage.mark_local_modified(B.storage.origin_slot)
        return B
    return redistribute(A, B)


def scale_row_col(equed, R, C, A, opts=None):
    """A = diag(R) A diag(C) (src/scale_row_col.cc); R, C are full-length
    vectors (global indexing) replicated on all ranks."""
    s, slot, lb = _bc_pieces(A, opts)
    bc = s.bc
    if lb.mloc and lb.nloc:
        dev = lb.data.device
        rdt = torch.float64 if lb.data.dtype in (torch.float64, torch.complex128) else torch.float32
        ridx = torch.tensor([l2g(lb.row_off + i, bc.mb, bc.pr, bc.p) - lb.grow0 for i in range(lb.mloc)])
        cidx = torch.tensor([l2g(lb.col_off + j, bc.nb, bc.pc, bc.q) - lb.gcol0 for j in range(lb.nloc)])
        r = torch.as_tensor(R, dtype=rdt)[ridx].to(dev) if R is not None else None
        c = torch.as_tensor(C, dtype=rdt)[cidx].to(dev) if C is not None else None
        ops.gescale_row_col(str(getattr(equed, "value", equed)), r, c, lb.data)
    s.mark_local_modified(slot)
    return A


# ------------------------------------------------------------------ norms
def norm(norm_type, A, opts=None, scope=NormScope.Matrix):
    """Matrix norm (Max / One / Inf / Fro) of a distributed matrix, with the
    matrix type's structure (general, trapezoid/triangular, symmetric/
    Hermitian with one stored triangle).  NaN propagates."""
    nt = Norm.from_string(norm_type) if not isinstance(norm_type, Norm) else norm_type
    s = A.storage
    band = hasattr(s, "in_window") and not (A.ioffset or A.joffset or A.row0_offset or A.col0_offset)
    if s.bc is None and not band:
        D = allgather_dense(A)
        return _dense_norm(nt, D, A)
    kind = _diag_kind(A)
    herm = kind in ("hermitian", "symmetric")
    hv = (2 if kind == "hermitian" and s.dtype.is_complex else 1) if herm else 0   # kernel flag
    diag = 'U' if getattr(A, "_diag", None) is not None and A._diag.value == 'U' and kind == "trapezoid" else 'N'
    # op: norms of A^T swap One <-> Inf
    if A.op() != Op.NoTrans and not herm:
        nt = {Norm.One: Norm.Inf, Norm.Inf: Norm.One}.get(nt, nt)
    comm = s.comm
    m_g, n_g = A._um(), A._un()
    if band:
        # compact band storage: the stored tiles (outside entries are zero)
        slot = s.band_slot()
        dev = s.get_slab(slot).device
        up = A.uploPhysical() if kind != "general" else None

        def pieces():
            for (i, j, sl) in list(s.tiles.keys()):
                if sl != slot or not s.tileIsLocal(i, j):
                    continue
                if up is not None and ((i < j) if up == Uplo.Lower else (i > j)):
                    continue
                r0, c0 = s.row_offsets[i], s.col_offsets[j]
                t = s.tiles[(i, j, sl)]
                u = up.value if (up is not None and i == j) else 'G'
                yield t, u, list(range(r0, r0 + t.shape[0])), list(range(c0, c0 + t.shape[1]))
        if A.op() != Op.NoTrans:
            m_g, n_g = n_g, m_g
    else:
        lb = A.local_block()
        dev = lb.data.device

        def pieces():
            if lb.mloc and lb.nloc and s.bc.pr >= 0:
                for blk, u in _local_uplo_blocks(A, lb):
                    gr, gc = _piece_globals(blk, lb)
                    yield blk, u, gr, gc
    rdt = torch.float64 if s.dtype in (torch.float64, torch.complex128) else torch.float32
    code = {Norm.Max: 'M', Norm.One: '1', Norm.Inf: 'I', Norm.Fro: 'F'}[nt]
    # every piece's per-column / per-row contributions come from the genorm
    # kernels; they are O(m + n) numbers, combined on the HOST (numpy) -- no
    # torch arithmetic on the device -- and reduced over the ranks as one
    # small device tensor (RCCL) per quantity
    colv = np.zeros(n_g, dtype=np.float64)
    rowv = np.zeros(m_g, dtype=np.float64)
    mx, fro2, nan = 0.0, 0.0, False
    for blk, u, gr, gc in pieces():
        on_diag = u != 'G'
        if herm and code in ('1', 'I'):
            if on_diag:
                c, r = ops.genorm_local('1', blk, uplo=u, herm=hv)
            else:
                c, _ = ops.genorm_local('1', blk)
                _, r = ops.genorm_local('I', blk)
            np.add.at(colv, np.asarray(gc), c.cpu().double().numpy())
            np.add.at(rowv, np.asarray(gr), r.cpu().double().numpy())
            continue
        c, r = ops.genorm_local(code, blk, uplo=u, diag=diag, herm=hv if on_diag else 0)
        if code == 'M':
            v = float(ops.genorm_local('M', c.view(-1, 1))[0][0]) if c.numel() else 0.0   # NaN propagates
            if v != v:
                nan = True
            else:
                mx = max(mx, v)
        elif code == 'F':
            ch = c.cpu().double().numpy()
            fro2 += float(np.sum(ch[:, 0] ** 2 * ch[:, 1])) * (2 if (herm and not on_diag) else 1)
        else:
            np.add.at(colv, np.asarray(gc), c.cpu().double().numpy())
            np.add.at(rowv, np.asarray(gr), r.cpu().double().numpy())

    def _reduce(x, op):
        if comm.size == 1:
            return x
        t = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64)).to(dev)
        comm.allreduce(t, op)
        return t.cpu().numpy()
    if code == 'M':
        out = _reduce(np.asarray([mx, 1.0 if nan else 0.0]), "max")
        return float("nan") if out[1] > 0 else float(out[0])
    if code == 'F':
        return float(np.sqrt(_reduce(np.asarray([fro2]), "sum")[0]))
    colv = _reduce(colv, "sum")
    rowv = _reduce(rowv, "sum")
    if herm:
        tot = colv + (rowv if m_g == n_g else 0)
        return float(tot.max()) if tot.size else 0.0
    if code == '1':
        return float(colv.max()) if colv.size else 0.0
    return float(rowv.max()) if rowv.size else 0.0


def _piece_globals(blk, lb):
    base = blk.storage_offset() - lb.data.storage_offset()
    ldd = max(1, lb.data.stride(1))
    lr, lc = base % ldd, base // ldd
    gr = [l2g(lb.row_off + lr + i, lb.mb, lb.pr, lb.p) - lb.grow0 for i in range(blk.shape[0])]
    gc = [l2g(lb.col_off + lc + j, lb.nb, lb.pc, lb.q) - lb.gcol0 for j in range(blk.shape[1])]
    return gr, gc


def _dense_norm(nt, D, A):
    """Norm of the gathered op(A) for storages without a 2D block-cyclic map,
    through the same genorm kernels as the distributed path (the stored
    triangle is masked inside the kernel, no dense rebuild)."""
    m, n = D.shape
    if not (m and n):
        return 0.0
    kind = _diag_kind(A)
    herm = kind in ("hermitian", "symmetric")
    u = 'G' if kind == "general" else A.uplo().value      # D is op(A): logical triangle
    hv = (2 if kind == "hermitian" and D.is_complex() else 1) if herm else 0
    diag = 'U' if getattr(A, "_diag", None) is not None and A._diag.value == 'U' and kind == "trapezoid" else 'N'
    code = {Norm.Max: 'M', Norm.One: '1', Norm.Inf: 'I', Norm.Fro: 'F'}[nt]
    if D.stride(0) != 1:
        # row-major D is the column-major D^T: same |entries| transposed, so
        # the stored triangle flips and One <-> Inf (|conj| = || for Hermitian)
        D = D.transpose(0, 1)
        u = {'L': 'U', 'U': 'L'}.get(u, u)
        code = {'1': 'I', 'I': '1'}.get(code, code)
    if herm and code in ('1', 'I'):
        c, r = ops.genorm_local('1', D, uplo=u, herm=hv)
        return float((c + r).max())
    c, r = ops.genorm_local(code, D, uplo=u, diag=diag, herm=hv)
    if code == 'M':
        return float("nan") if bool(torch.isnan(c).any()) else float(c.max())
    if code == 'F':
        return float(torch.sqrt((c[:, 0] ** 2 * c[:, 1]).sum()))
    return float(c.max()) if code == '1' else float(r.max())


def colNorms(norm_type, A, opts=None):
    """Per-column norms (Max only, like SLATE `colNorms`, src/colNorms.cc)."""
    s = A.storage
    lb = A.local_block()
    rdt = torch.float64 if s.dtype in (torch.float64, torch.complex128) else torch.float32
    n_g = A._un()
    colv = torch.zeros(n_g, dtype=rdt, device=lb.data.device)
    if lb.mloc and lb.nloc:
        c, _ = ops.genorm_local('M', lb.data)
        gc = [l2g(lb.col_off + j, lb.nb, lb.pc, lb.q) - lb.gcol0 for j in range(lb.nloc)]
        gc_t = torch.as_tensor(gc, device=colv.device)
        colv.index_put_((gc_t,), torch.maximum(colv[gc_t], c))
    if s.comm.size > 1:
        s.comm.allreduce(colv, "max")
    return colv


def set_lambda(fn, A, opts=None):
    """A(i, j) = fn(i, j) for every stored element (src/set_lambdas.cc);
    fn receives broadcastable global index tensors (rows[:, None],
    cols[None, :]) and must return a tensor (or scalar)."""
    s, slot, lb = _bc_pieces(A, opts)
    if lb.mloc and lb.nloc:
        dev = lb.data.device
        gr = torch.tensor([lb.global_row(i) for i in range(lb.mloc)], device=dev)[:, None]
        gc = torch.tensor([lb.global_col(j) for j in range(lb.nloc)], device=dev)[None, :]
        v = fn(gr, gc)
        v = torch.as_tensor(v, device=dev).to(lb.data.dtype).expand(lb.mloc, lb.nloc)
        up = A.uploPhysical()
        if up == Uplo.Lower:
            keep = gr >= gc
        elif up == Uplo.Upper:
            keep = gr <= gc
        else:
            keep = None
        if keep is None:
            lb.data.copy_(v)
        else:
            lb.data.copy_(torch.where(keep, v, lb.data))
    s.mark_local_modified(slot)
    return A
