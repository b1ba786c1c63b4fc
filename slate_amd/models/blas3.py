"""Parallel BLAS-3: gemm, hemm/symm, herk/syrk, her2k/syr2k, trmm, trsm.

Reference: `src/gemm.cc` (method select), `src/gemmC.cc:39-202` (SUMMA,
stationary C, listBcastMT of A(:,k) / B(k,:)), `src/gemmA.cc`,
`src/herk.cc`, `src/syrk.cc`, `src/her2k.cc`, `src/syr2k.cc`,
`src/hemm*.cc`, `src/symm.cc`, `src/trmm.cc`, `src/trsm*.cc`,
`src/work/work_trsm.cc:102-265`.

MI355X design:
* one rank (p = q = 1, the common single-GPU case): each routine is ONE
  call of the tile-level op on the whole local matrix (MFMA GEMM, masked
  GEMM for herk/her2k, blocked LDS+GEMM trsm/trmm) -- no tile loops;
* p x q ranks: SUMMA with one row-communicator broadcast of the A panel
  and one column-communicator broadcast of the B panel per k-step, the
  broadcast of step k+1 issued on the high-priority stream while the
  local GEMM of step k runs on the low-priority stream (SLATE gemmC
  lookahead), herk with the potrf-style panel/transposed-panel assembly,
  trsm with batched point-to-point tile delivery (tilecomm.exchange_tiles).
"""
from __future__ import annotations

import torch

from .. import ops
from ..core.enums import Diag, MethodGemm, Op, Option, Side, Uplo
from ..core.exceptions import SlateError
from ..core.options import get_option
from ..core.storage import DEV, l2g
from ..parallel.streams import StreamSet
from ..parallel.tilecomm import exchange_tiles
from ..utils.trace import trace_block
from ._util import conj_trans, grid_of, target_slot, tiles_local_before


def _single(*mats):
    return all(M.storage.comm.size == 1 or (M.storage.bc is not None and M.storage.bc.p * M.storage.bc.q == 1)
               for M in mats) and all(M.storage.bc is not None for M in mats)


def _loc(X, slot=None):
    lb = X.local_block(slot)
    return lb.data, X.op().value, lb


def _done(*mats):
    for M in mats:
        M.storage.mark_local_modified(M.storage.origin_slot)


def _dense(X):
    from .aux import allgather_dense
    return allgather_dense(X)


def _dense_store(X, D):
    from .aux import from_dense
    from_dense(X, D)


def _full_herm(D, uplo, herm=True):
    L = torch.tril(D) if uplo == Uplo.Lower else torch.triu(D)
    Dg = torch.diagonal(L)
    F = L + (L.transpose(0, 1).conj() if herm else L.transpose(0, 1)) - torch.diag(Dg)
    if herm and D.dtype.is_complex:
        F.diagonal().imag.zero_()
    return F


# ------------------------------------------------------------------- gemm
def gemm(alpha, A, B, beta, C, opts=None):
    """C = alpha op(A) op(B) + beta C."""
    if C.op() != Op.NoTrans:
        # C^T = op(B)^T op(A)^T
        t = (lambda X: X.transpose()) if C.op() == Op.Trans else (lambda X: X.conj_transpose())
        if C.op() == Op.ConjTrans:
            alpha, beta = complex(alpha).conjugate(), complex(beta).conjugate()
        return gemm(alpha, t(B), t(A), beta, t(C), opts)
    with trace_block("gemm"):
        if _single(A, B, C):
            a, ta, _ = _loc(A)
            b, tb, _ = _loc(B)
            c, _, _ = _loc(C)
            ops.gemm(alpha, a, b, beta, c, ta, tb)
            _done(C)
            return C
        return _gemm_summa(alpha, A, B, beta, C, opts)


def _aligned(A, B, C):
    """SUMMA fast path: same grid & tile size, NoTrans, tile-aligned views,
    A's rows aligned with C's rows and B's columns with C's columns."""
    sA, sB, sC = A.storage.bc, B.storage.bc, C.storage.bc
    if None in (sA, sB, sC) or A.op() != Op.NoTrans or B.op() != Op.NoTrans:
        return False
    if not (A.storage.local and B.storage.local and C.storage.local):
        return False
    if (sA.p, sA.q, sA.order) != (sC.p, sC.q, sC.order) or (sB.p, sB.q, sB.order) != (sC.p, sC.q, sC.order):
        return False
    if len({sA.mb, sA.nb, sB.mb, sB.nb, sC.mb, sC.nb}) != 1:
        return False
    rA, cA = A.global_offsets()
    rB, cB = B.global_offsets()
    rC, cC = C.global_offsets()
    nb = sC.nb
    return rA == rC and cB == cC and all(x % nb == 0 for x in (cA, rB, rC, cC))


def _gemm_summa(alpha, A, B, beta, C, opts):
    if not _aligned(A, B, C):
        # general distributions / transposed operands: gather-compute-scatter
        Da, Db, Dc = _dense(A), _dense(B), _dense(C)
        ops.gemm(alpha, ops.as_colmajor(Da), ops.as_colmajor(Db), beta, Dc_ := ops.as_colmajor(Dc.clone()))
        _dense_store(C, Dc_)
        return C
    s = C.storage
    bc = s.bc
    grid = grid_of(C)
    slot = target_slot(C, opts)
    la_ = A.local_block(slot)
    lb_ = B.local_block(slot)
    lc_ = C.local_block(slot)
    dev = lc_.data.device
    nb, p, q, pr, pc = bc.nb, bc.p, bc.q, bc.pr, bc.pc
    rA0, cA0 = A.global_offsets()
    rB0, _ = B.global_offsets()
    kt = A.nt()
    ss = StreamSet(dev, reserve_cus=0)
    ss.fork()
    la = max(0, int(get_option(opts, Option.Lookahead, 1)))
    panels = {}

    def bcast_step(k):
        gA = cA0 // nb + k          # storage tile column of A
        gB = rB0 // nb + k          # storage tile row of B
        kb = min(nb, A._un() - k * nb)
        mloc, nloc = lc_.mloc, lc_.nloc
        # A panel: local rows x kb from owner process column
        Ap = ops.colmajor_empty(mloc, kb, s.dtype, dev)
        if gA % q == pc and mloc:
            lc = tiles_local_before(gA, q, pc) * nb - la_.col_off
            Ap.copy_(la_.data[:, lc:lc + kb])
        if mloc:
            grid.row_comm.bcast(Ap, gA % q)
        Bp = ops.colmajor_empty(kb, nloc, s.dtype, dev)
        if gB % p == pr and nloc:
            lr = tiles_local_before(gB, p, pr) * nb - lb_.row_off
            Bp.copy_(lb_.data[lr:lr + kb, :])
        if nloc:
            grid.col_comm.bcast(Bp, gB % p)
        return Ap, Bp

    with ss.use(ss.panel):
        for k in range(min(la + 1, kt)):
            panels[k] = (bcast_step(k), ss.event(ss.panel))
    for k in range(kt):
        (Ap, Bp), ev = panels.pop(k)
        us = ss.update[0]
        with ss.use(us):
            ss.wait(us, ev)
            if Ap.is_cuda:
                Ap.record_stream(us)
                Bp.record_stream(us)
            if lc_.mloc and lc_.nloc:
                ops.gemm(alpha, Ap, Bp, beta if k == 0 else 1.0, lc_.data)
        if k + la + 1 < kt:
            with ss.use(ss.panel):
                panels[k + la + 1] = (bcast_step(k + la + 1), ss.event(ss.panel))
    if kt == 0 and lc_.mloc and lc_.nloc:
        ops.gescale(beta, lc_.data)
    ss.join()
    _done(C)
    return C


def multiply(alpha, A, B, beta, C, opts=None):
    """Simplified-API name (include/slate/simplified_api.hh)."""
    if getattr(A, "_kind", "") in ("hermitian", "symmetric"):
        return hemm(Side.Left, alpha, A, B, beta, C, opts) if A._kind == "hermitian" else \
            symm(Side.Left, alpha, A, B, beta, C, opts)
    if getattr(B, "_kind", "") in ("hermitian", "symmetric"):
        return hemm(Side.Right, alpha, B, A, beta, C, opts) if B._kind == "hermitian" else \
            symm(Side.Right, alpha, B, A, beta, C, opts)
    return gemm(alpha, A, B, beta, C, opts)


# ---------------------------------------------------------------- herk etc.
def herk(alpha, A, beta, C, opts=None, _sym=False):
    """C = alpha op(A) op(A)^H + beta C, C Hermitian (stored triangle only)."""
    with trace_block("syrk" if _sym else "herk"):
        if _single(A, C):
            a, ta, _ = _loc(A)
            c, _, lbc = _loc(C)
            up = 'L' if C.uploPhysical() == Uplo.Lower else 'U'
            if ta == 'N':
                (ops.syrk if _sym else ops.herk)(up, 'N', alpha, a, beta, c)
            else:
                (ops.syrk if _sym else ops.herk)(up, 'C' if not _sym else 'T', alpha, a, beta, c)
            _done(C)
            return C
        Da = _dense(A)
        Dc = _dense(C)
        t = Da @ (Da.transpose(0, 1) if _sym else Da.transpose(0, 1).conj())
        R = alpha * t + beta * Dc
        tri = torch.tril if C.uploPhysical() == Uplo.Lower else torch.triu
        R = tri(R) + (Dc - tri(Dc))
        _dense_store(C, R)
        return C


def syrk(alpha, A, beta, C, opts=None):
    return herk(alpha, A, beta, C, opts, _sym=True)


def her2k(alpha, A, B, beta, C, opts=None, _sym=False):
    """C = alpha op(A) op(B)^H + conj(alpha) op(B) op(A)^H + beta C."""
    with trace_block("her2k"):
        if _single(A, B, C):
            a, ta, _ = _loc(A)
            b, tb, _ = _loc(B)
            c, _, _ = _loc(C)
            up = 'L' if C.uploPhysical() == Uplo.Lower else 'U'
            fn = ops.syr2k if _sym else ops.her2k
            fn(up, 'N' if ta == 'N' else ('T' if _sym else 'C'), alpha, a, b, beta, c)
            _done(C)
            return C
        Da, Db, Dc = _dense(A), _dense(B), _dense(C)
        H = (lambda X: X.transpose(0, 1)) if _sym else (lambda X: X.transpose(0, 1).conj())
        a2 = alpha if _sym else complex(alpha).conjugate()
        R = alpha * (Da @ H(Db)) + a2 * (Db @ H(Da)) + beta * Dc
        tri = torch.tril if C.uploPhysical() == Uplo.Lower else torch.triu
        R = tri(R) + (Dc - tri(Dc))
        _dense_store(C, R)
        return C


def syr2k(alpha, A, B, beta, C, opts=None):
    return her2k(alpha, A, B, beta, C, opts, _sym=True)


def hemm(side, alpha, A, B, beta, C, opts=None, _sym=False):
    """C = alpha A B + beta C (Left) or alpha B A + beta C (Right), A Hermitian."""
    side = Side.from_string(side) if not isinstance(side, Side) else side
    with trace_block("symm" if _sym else "hemm"):
        if _single(A, B, C):
            a, _, _ = _loc(A)
            b, tb, _ = _loc(B)
            c, _, _ = _loc(C)
            n = a.shape[0]
            F = ops.colmajor_empty(n, n, a.dtype, a.device)
            up = 'L' if A.uploPhysical() == Uplo.Lower else 'U'
            other = 'U' if up == 'L' else 'L'
            ops.gecopy(a, F, uplo=up)
            ops.gecopy(a, F, uplo=other, trans='T' if _sym else 'C')
            if not _sym and a.dtype.is_complex:
                # diagonal of a Hermitian matrix is real
                d = torch.diagonal(F)
                d.copy_(d.real.to(F.dtype))
            if side == Side.Left:
                ops.gemm(alpha, F, b, beta, c, 'N', tb)
            else:
                ops.gemm(alpha, b, F, beta, c, tb, 'N')
            _done(C)
            return C
        Fa = _full_herm(_dense(A), A.uploPhysical(), herm=not _sym)
        Db, Dc = _dense(B), _dense(C)
        R = alpha * (Fa @ Db if side == Side.Left else Db @ Fa) + beta * Dc
        _dense_store(C, R)
        return C


def symm(side, alpha, A, B, beta, C, opts=None):
    return hemm(side, alpha, A, B, beta, C, opts, _sym=True)


# -------------------------------------------------------------- trmm / trsm
def _tri_args(A):
    uplo = 'L' if A.uploPhysical() == Uplo.Lower else 'U'
    diag = A.diag().value if hasattr(A, "diag") else 'N'
    return uplo, diag


def trmm(side, alpha, A, B, opts=None):
    """B = alpha op(A) B (Left) or alpha B op(A) (Right), A triangular."""
    side = Side.from_string(side) if not isinstance(side, Side) else side
    with trace_block("trmm"):
        if _single(A, B) and B.op() == Op.NoTrans:
            a, ta, _ = _loc(A)
            b, _, _ = _loc(B)
            uplo, diag = _tri_args(A)
            ops.trmm(side.value, uplo, ta, diag, alpha, a, b)
            _done(B)
            return B
        Da = _dense(A)
        uplo, diag = A.uploPhysical(), A.diag()
        # op(A) as a dense logical matrix: _dense already applies op;
        # the stored triangle of op(A) is the logical triangle
        tri = torch.tril if A.uploLogical() == Uplo.Lower else torch.triu
        T = tri(Da)
        if diag == Diag.Unit:
            T = T - torch.diag(torch.diagonal(T)) + torch.eye(T.shape[0], dtype=T.dtype, device=T.device)
        Db = _dense(B)
        R = alpha * (T @ Db if side == Side.Left else Db @ T)
        _dense_store(B, R)
        return B


def trsm(side, alpha, A, B, opts=None):
    """Solve op(A) X = alpha B (Left) or X op(A) = alpha B (Right); B <- X."""
    side = Side.from_string(side) if not isinstance(side, Side) else side
    with trace_block("trsm"):
        if _single(A, B) and B.op() == Op.NoTrans:
            a, ta, _ = _loc(A)
            b, _, _ = _loc(B)
            uplo, diag = _tri_args(A)
            ops.trsm(side.value, uplo, ta, diag, alpha, a, b)
            _done(B)
            return B
        if side == Side.Left and B.op() == Op.NoTrans and A.storage.bc is not None and B.storage.bc is not None:
            return _trsm_left_dist(alpha, A, B, opts)
        # Right side (or transposed B): X op(A) = B  <=>  op(A)^H X^H = B^H
        Da = _dense(A)
        tri = torch.tril if A.uploLogical() == Uplo.Lower else torch.triu
        T = tri(Da)
        if A.diag() == Diag.Unit:
            T = T - torch.diag(torch.diagonal(T)) + torch.eye(T.shape[0], dtype=T.dtype, device=T.device)
        Db = _dense(B)
        Tm = ops.as_colmajor(T.clone())
        X = ops.as_colmajor((alpha * Db).clone())
        ops.trsm(side.value, 'L' if A.uploLogical() == Uplo.Lower else 'U', 'N', 'N', 1.0, Tm, X)
        _dense_store(B, X)
        return B


def _trsm_left_dist(alpha, A, B, opts):
    """Distributed Left trsm, any uplo/op of A (work::trsm analogue):
    per tile row k: diag tile -> owners of B(k,:), local solve, X(k,:) down
    each process column, A(:,k) panel tiles delivered to the owners of the
    B rows they update (batched p2p), one local GEMM."""
    sB = B.storage
    bcB = sB.bc
    comm = sB.comm
    grid = grid_of(B)
    slot = target_slot(B, opts)
    lbB = B.local_block(slot)
    dev = lbB.data.device
    nb, p, q, pr, pc = bcB.nb, bcB.p, bcB.q, bcB.pr, bcB.pc
    uplo_l = A.uploLogical()
    lower = uplo_l == Uplo.Lower
    diag = A.diag().value
    opA = A.op()
    mt = B.mt()
    rB0, _ = B.global_offsets()
    if rB0 % nb:
        raise SlateError("trsm: B must start on a tile boundary")
    gb0 = rB0 // nb
    if alpha != 1 and lbB.mloc and lbB.nloc:
        ops.gescale(alpha, lbB.data)
    order = range(mt) if lower else range(mt - 1, -1, -1)

    def stored_key(i, k):
        # view tile (i,k) of op(A) -> stored tile (global indices)
        gi, gj = A._global_ij(i, k)
        return (gi, gj)

    def owner(key):
        return A.storage.tileRank(key)

    def get_tile(key):
        sA = A.storage
        return sA.tile_data(key[0], key[1], sA.origin_slot)

    def shape(key):
        sA = A.storage
        return sA.tileMb(key[0]), sA.tileNb(key[1])

    for k in order:
        gk = gb0 + k
        kb = B.tileMb(k)
        # rows of B updated by step k
        rows = [i for i in (range(k + 1, mt) if lower else range(0, k))]
        # who needs what: diag tile -> process row of B(k,:); panel tile (i,k) -> process row of B(i,:)
        needs = {}
        for r in range(comm.size):
            rpr, rpc = grid.coords(r)
            ks = []
            if (gk % p) == rpr:
                ks.append(stored_key(k, k))
            ks += [stored_key(i, k) for i in rows if ((gb0 + i) % p) == rpr]
            needs[r] = ks
        got = exchange_tiles(comm, needs, owner, get_tile, shape, sB.dtype, dev)
        # local solve on B(k,:) local columns
        Xk = ops.colmajor_empty(kb, lbB.nloc, sB.dtype, dev)
        if (gk % p) == pr and lbB.nloc:
            lr = tiles_local_before(gk, p, pr) * nb - lbB.row_off
            Bk = lbB.data[lr:lr + kb, :]
            Dk = got[stored_key(k, k)]
            ops.trsm('L', A.uploPhysical().value[0] if hasattr(A.uploPhysical(), "value") else 'L',
                     opA.value, diag, 1.0, Dk, Bk)
            Xk.copy_(Bk)
        if lbB.nloc:
            grid.col_comm.bcast(Xk, gk % p) if p > 1 else None
        # panel for my local rows that are updated
        my_rows = [i for i in rows if ((gb0 + i) % p) == pr]
        if my_rows and lbB.nloc:
            # local rows of those tiles form contiguous groups; do one GEMM per tile row
            for i in my_rows:
                t = got[stored_key(i, k)]
                lr = tiles_local_before(gb0 + i, p, pr) * nb - lbB.row_off
                mi = B.tileMb(i)
                ops.gemm(-1.0, t, Xk, 1.0, lbB.data[lr:lr + mi, :], opA.value, 'N')
    _done(B)
    return B


def triangular_multiply(alpha, A, B, opts=None):
    return trmm(Side.Left, alpha, A, B, opts)


def triangular_solve(alpha, A, B, opts=None):
    return trsm(Side.Left, alpha, A, B, opts)


def rank_k_update(alpha, A, beta, C, opts=None):
    return herk(alpha, A, beta, C, opts) if getattr(C, "_kind", "") == "hermitian" else syrk(alpha, A, beta, C, opts)


def rank_2k_update(alpha, A, B, beta, C, opts=None):
    return her2k(alpha, A, B, beta, C, opts) if getattr(C, "_kind", "") == "hermitian" else \
        syr2k(alpha, A, B, beta, C, opts)
