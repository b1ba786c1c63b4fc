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
from ._panels import assemble_cols, plan_col_gather, row_bcast
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


def _grid_params(X):
    """(mb, nb, p, q, order) of X's block-cyclic grid, or a default grid."""
    bc = X.storage.bc
    if bc is not None:
        return bc.mb, bc.nb, bc.p, bc.q, bc.order
    from ..core import func
    from ..core.enums import GridOrder
    nb = max(1, X.storage.tileMb(0) if X.storage.mt else 1)
    p, q = func.grid_shape(X.storage.comm.size)
    return nb, nb, p, q, GridOrder.Col


def _fresh(like, m, n, slot, dtype=None, cls=None, uplo=None):
    """A new allocated block-cyclic m x n matrix on ``like``'s grid."""
    from ..core.matrix import HermitianMatrix, Matrix
    mb, nb, p, q, order = _grid_params(like)
    s = like.storage
    dt = dtype or s.dtype
    if cls is not None and uplo is not None:
        from ..core.storage import MatrixStorage
        from ..core import func
        st = MatrixStorage(m, n, func.uniform_blocksize(m, mb), func.uniform_blocksize(n, nb),
                           func.process_2d_grid(order, p, q), s.comm, dt, s.device)
        M = cls(uplo, _storage=st)
    else:
        M = Matrix(m, n, nb=nb, mb=mb, p=p, q=q, comm=s.comm, dtype=dt, device=s.device, order=order)
    M.insertLocalTiles(device=s.device if slot == DEV else -1)
    return M


def _copy_in(X, like, slot, uplo=None):
    """Fresh block-cyclic copy of the logical matrix op(X) on like's grid."""
    from ..parallel.redist import redistribute_pieces
    F = _fresh(like, X.m(), X.n(), slot, X.storage.dtype)
    redistribute_pieces(X, F, uplo=uplo)
    return F


def _copy_out(F, X, uplo=None):
    from ..parallel.redist import redistribute_pieces
    redistribute_pieces(F, X, uplo=uplo)


def _same_grid(X, C):
    a, c = X.storage.bc, C.storage.bc
    return a is not None and c is not None and bool(X.storage.local) and \
        (a.p, a.q, a.order, a.mb, a.nb) == (c.p, c.q, c.order, c.mb, c.nb) and a.mb == a.nb


def _rows_aligned(A, C):
    """op(A) = A, same grid, A's rows start where C's rows start, A's
    columns start on a tile boundary."""
    if A.op() != Op.NoTrans or not _same_grid(A, C):
        return False
    rA, cA = A.global_offsets()
    rC, _ = C.global_offsets()
    nb = C.storage.bc.nb
    return rA == rC and cA % nb == 0


def _cols_aligned(B, C):
    if B.op() != Op.NoTrans or not _same_grid(B, C):
        return False
    rB, cB = B.global_offsets()
    _, cC = C.global_offsets()
    return cB == cC and rB % C.storage.bc.nb == 0


def _at_origin(C):
    return C.storage.bc is not None and bool(C.storage.local) and C.global_offsets() == (0, 0) \
        and C.op() == Op.NoTrans and C.storage.bc.mb == C.storage.bc.nb


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
        return _gemm_dist(alpha, A, B, beta, C, opts)


def _gemm_method(B, opts):
    """src/gemm.cc:11-24: stationary A when B has a single block column
    (one process per GPU here, so the reference's multi-GPU exception does
    not apply)."""
    m = get_option(opts, Option.MethodGemm, MethodGemm.Auto)
    if m in (MethodGemm.A, MethodGemm.C):
        return m
    return MethodGemm.A if B.nt() < 2 else MethodGemm.C


def _gemm_dist(alpha, A, B, beta, C, opts):
    """Distributed gemm on any distributions / ops: operands that are not
    already aligned with C's grid are redistributed (one batched p2p
    exchange each, parallel/redist.py) -- never gathered."""
    slot = target_slot(C, opts)
    work = C
    if not (_rows_aligned(A, C) and _cols_aligned(B, C)) and not _at_origin(C):
        work = _fresh(C, C.m(), C.n(), slot)
        if beta != 0:
            _copy_out(C, work)
    Aw = A if _rows_aligned(A, work) else _copy_in(A, work, slot)
    Bw = B if _cols_aligned(B, work) else _copy_in(B, work, slot)
    if _gemm_method(Bw, opts) == MethodGemm.A:
        _gemmA(alpha, Aw, Bw, beta, work, opts)
    else:
        _gemm_summa(alpha, Aw, Bw, beta, work, opts)
    if work is not C:
        _copy_out(work, C)
    return C


def _gemmA(alpha, A, B, beta, C, opts):
    """Stationary-A gemm (src/gemmA.cc, listReduce of partial C tiles):
    for each block column jb of C, B(:, jb) is delivered to the owners of
    the matching columns of A, each rank multiplies its local A block, and
    the partial products are reduced over the process row onto the owner of
    C(:, jb).  A never moves -- the right choice when B/C are skinny."""
    if A.global_offsets()[1] != 0 or B.global_offsets()[0] != 0:
        slot = target_slot(C, opts)
        A = A if A.global_offsets()[1] == 0 else _copy_in(A, C, slot)
        B = B if B.global_offsets()[0] == 0 else _copy_in(B, C, slot)
    s = C.storage
    bc = s.bc
    grid = grid_of(C)
    slot = target_slot(C, opts)
    la_ = A.local_block(slot)
    lb_ = B.local_block(slot)
    lc_ = C.local_block(slot)
    dev = lc_.data.device
    nb, p, q, pr, pc = bc.nb, bc.p, bc.q, bc.pr, bc.pc
    kt = A.nt()
    plan = plan_col_gather(B.storage.tileMb, 0, kt, nb, p, q, pc, dev)
    _, cB0 = B.global_offsets()
    for jb in range(C.nt()):
        gj = cB0 // nb + jb
        owner = gj % q
        wb = C.tileNb(jb)
        # B(:, jb) local rows -> every rank of this process row
        lcb = tiles_local_before(gj, q, pc) * nb - lb_.col_off
        src = lb_.data[:, lcb:lcb + wb] if pc == owner else None
        Prow = row_bcast(grid, src, owner, lb_.mloc, wb, s.dtype, dev)
        # rows of B(:, jb) matching my local columns of A
        Bq = assemble_cols(plan, Prow, grid, p, wb, s.dtype, dev)
        P = ops.colmajor_zeros(la_.mloc, wb, s.dtype, dev)
        if la_.mloc and la_.nloc:
            ops.gemm(alpha, la_.data, Bq, 0.0, P)
        if q > 1 and la_.mloc:
            grid.row_comm.reduce(P, owner)
        if pc == owner and lc_.mloc:
            lcc = tiles_local_before(gj, q, pc) * nb - lc_.col_off
            if beta == 0:
                ops.gecopy(P, lc_.data[:, lcc:lcc + wb])     # C is not read when beta = 0
            else:
                ops.geadd(1.0, P, beta, lc_.data[:, lcc:lcc + wb])
    _done(C)
    return C


def _gemm_summa(alpha, A, B, beta, C, opts):
    """SUMMA, stationary C (src/gemmC.cc:39-202) on aligned operands."""
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
def _diag_aligned(C):
    """C is a whole-tile diagonal block of a block-cyclic square storage."""
    s = C.storage
    return s.bc is not None and bool(s.local) and C.op() == Op.NoTrans and C.ioffset == C.joffset \
        and C.row0_offset == 0 and C.col0_offset == 0 and C.last_mb is None and C.last_nb is None \
        and s.bc.mb == s.bc.nb and s.m == s.n


def _herm_work(C, slot):
    """(work matrix, needs copy-back): a diagonal-aligned Hermitian work
    view for the rank-k kernels."""
    if _diag_aligned(C):
        return C, False
    from ..core.matrix import HermitianMatrix
    W = _fresh(C, C.n(), C.n(), slot, cls=HermitianMatrix, uplo=C.uplo())
    _copy_out(C, W, uplo=C.uplo())
    return W, True


def _rank_k_dist(alpha, pairs, beta, C, opts, sym):
    """C = beta C + sum over (alpha_i, X_i, Y_i) of alpha_i X_i Y_i^H (^T if
    sym), only C's stored triangle.  Per block column k of the X_i:
    Prow(X_i) along the process row, Lcol(Y_i) down the process column
    (potrf-style panel assembly, _panels.py), one masked MFMA GEMM each --
    SLATE internal_herk.cc:350-535 / internal_her2k.cc, without the
    per-tile batches."""
    slot = target_slot(C, opts)
    W, back = _herm_work(C, slot)
    s = W.storage
    bc = s.bc
    grid = grid_of(W)
    lbC = W.local_block(slot)
    dev = lbC.data.device
    nb, p, q, pr, pc = bc.nb, bc.p, bc.q, bc.pr, bc.pc
    ct = 'T' if sym else conj_trans(s.dtype)
    lower = W.uplo() == Uplo.Lower
    mask = lbC.mask(1 if lower else 2)
    g0, nt = W.ioffset, W.mt()
    ops_ = []
    for (al, X, Y) in pairs:
        Xw = X if _rows_aligned(X, W) else _copy_in(X, W, slot)
        Yw = Xw if Y is X else (Y if _rows_aligned(Y, W) else _copy_in(Y, W, slot))
        ops_.append((al, Xw, Yw))
    kt = ops_[0][1].nt() if ops_ else 0
    if kt == 0 or all(a == 0 for a, _, _ in ops_):
        if beta != 1:
            from .aux import scale
            scale(beta, 1.0, W)
    else:
        plan = plan_col_gather(s.tileMb, g0, g0 + nt, nb, p, q, pc, dev)
        first = True
        for kk in range(kt):
            panels = {}
            for (al, Xw, Yw) in ops_:
                for M in (Xw, Yw):
                    if id(M) in panels:
                        continue
                    lm = M.local_block(slot)
                    gk = M.global_offsets()[1] // nb + kk
                    kb = M.tileNb(kk)
                    lc = tiles_local_before(gk, q, pc) * nb - lm.col_off
                    src = lm.data[:, lc:lc + kb] if gk % q == pc else None
                    Prow = row_bcast(grid, src, gk % q, lm.mloc, kb, s.dtype, dev)
                    Lcol = assemble_cols(plan, Prow, grid, p, kb, s.dtype, dev)
                    panels[id(M)] = (Prow, Lcol)
            for (al, Xw, Yw) in ops_:
                Prow, _ = panels[id(Xw)]
                _, Lcol = panels[id(Yw)]
                if lbC.mloc and lbC.nloc:
                    ops.gemm(al, Prow, Lcol, beta if first else 1.0, lbC.data, 'N', ct, mask)
                first = False
    _done(W)
    if back:
        _copy_out(W, C, uplo=C.uplo())
    return C


def _real_diag(C, sym):
    """zherk/zher2k semantics: the diagonal of the Hermitian result is real."""
    if not sym and C.storage.dtype.is_complex and C.storage.bc is not None:
        from .aux import set_diag_imag_zero
        set_diag_imag_zero(C)
    return C


def _herm_base(C):
    """herk/her2k act on the stored Hermitian matrix: a (conj-)transposed
    Hermitian view is the same logical matrix."""
    if C.op() == Op.NoTrans:
        return C
    return C.conj_transpose() if C.op() == Op.ConjTrans else C.transpose()


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
            return _real_diag(C, _sym)
        _rank_k_dist(alpha, [(alpha, A, A)], beta, _herm_base(C), opts, _sym)
        return _real_diag(C, _sym)


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
            return _real_diag(C, _sym)
        a2 = alpha if _sym else complex(alpha).conjugate()
        if not C.storage.dtype.is_complex:
            a2 = float(complex(a2).real)
        _rank_k_dist(alpha, [(alpha, A, B), (a2, B, A)], beta, _herm_base(C), opts, _sym)
        return _real_diag(C, _sym)


def syr2k(alpha, A, B, beta, C, opts=None):
    return her2k(alpha, A, B, beta, C, opts, _sym=True)


def _full_from_stored(A, slot, herm=True):
    """General block-cyclic copy of a Hermitian/symmetric matrix with both
    triangles filled: the mirrored triangle by one transposing
    redistribution, the stored one (incl. the diagonal) on top."""
    from ..parallel.redist import redistribute_pieces
    n = A.n()
    F = _fresh(A, n, n, slot)
    u = A.uplo()
    other = Uplo.Upper if u == Uplo.Lower else Uplo.Lower
    H = A.conj_transpose() if herm else A.transpose()
    redistribute_pieces(H, F, uplo=other)
    redistribute_pieces(A, F, uplo=u)
    if herm and F.storage.dtype.is_complex:
        from .aux import set_diag_imag_zero
        set_diag_imag_zero(F)
    return F


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
        # hemmC with both triangles materialised once (SLATE broadcasts A
        # and A^H tiles per step and runs the diagonal tiles on the host,
        # src/hemmC.cc:147-429): one transposing redistribution, then SUMMA
        F = _full_from_stored(A, target_slot(C, opts), herm=not _sym)
        if side == Side.Left:
            return gemm(alpha, F, B, beta, C, opts)
        return gemm(alpha, B, F, beta, C, opts)


def symm(side, alpha, A, B, beta, C, opts=None):
    return hemm(side, alpha, A, B, beta, C, opts, _sym=True)


# -------------------------------------------------------------- trmm / trsm
def _tri_args(A):
    uplo = 'L' if A.uploPhysical() == Uplo.Lower else 'U'
    diag = A.diag().value if hasattr(A, "diag") else 'N'
    return uplo, diag


def _tri_as_general(A, slot):
    """op(A) of a triangular view as a general block-cyclic matrix with
    explicit zeros outside the triangle (unit diagonal materialised)."""
    from ..parallel.redist import redistribute_pieces
    n = A.n()
    F = _fresh(A, n, n, slot)           # zero-initialised
    redistribute_pieces(A, F, uplo=A.uplo())
    if A.diag() == Diag.Unit:
        from .aux import set_diag
        set_diag(F, 1.0)
    return F


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
        # distributed (work::trmm analogue): the triangle as a general
        # operand with zeros, one SUMMA product into a work matrix
        slot = target_slot(B, opts)
        T = _tri_as_general(A, slot)
        X = _fresh(B, B.m(), B.n(), slot)
        if side == Side.Left:
            gemm(alpha, T, B, 0.0, X, opts)
        else:
            gemm(alpha, B, T, 0.0, X, opts)
        _copy_out(X, B)
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
        slot = target_slot(B, opts)
        if side == Side.Right:
            # X op(A) = alpha B  <=>  op(A)^H X^H = conj(alpha) B^H  (^T when
            # op(A) = A^T): one transposing redistribution each way
            use_h = A.op() != Op.Trans
            tr = (lambda X: X.conj_transpose()) if use_h else (lambda X: X.transpose())
            Bw = B if B.op() == Op.NoTrans else _copy_in(B, B, slot)
            Bt = _copy_in(tr(Bw), Bw, slot)
            a2 = complex(alpha).conjugate() if (use_h and B.storage.dtype.is_complex) else alpha
            _trsm_left(a2, tr(A), Bt, slot)
            _copy_out(tr(Bt), B)
            return B
        if B.op() != Op.NoTrans or B.storage.bc is None or not B.storage.local \
                or B.global_offsets()[0] % B.storage.bc.nb:
            Bw = _copy_in(B, B, slot)
            _trsm_left(alpha, A, Bw, slot)
            _copy_out(Bw, B)
            return B
        return _trsm_left(alpha, A, B, slot)


def _trsm_left(alpha, A, B, slot):
    """Left solve on a block-cyclic NoTrans B whose rows start on a tile
    boundary; A is redistributed onto B's grid when its tiles do not match
    B's row tiles (stored triangle only)."""
    nb = B.storage.bc.nb
    sA = A.storage
    ok = sA.bc is not None and sA.bc.mb == nb and sA.bc.nb == nb and \
        all(x % nb == 0 for x in A.global_offsets()) and A.last_mb is None and A.last_nb is None
    if not ok:
        from ..core.matrix import TriangularMatrix
        F = _fresh(B, A.m(), A.n(), slot)
        from ..parallel.redist import redistribute_pieces
        redistribute_pieces(A, F, uplo=A.uplo())
        A = TriangularMatrix(A.uplo(), F, diag=A.diag())
    return _trsm_left_dist(alpha, A, B, slot)


def _trsm_left_dist(alpha, A, B, slot):
    """Distributed Left trsm, any uplo/op of A (work::trsm analogue,
    src/work/work_trsm.cc:102-265): per tile row k the diagonal tile goes to
    the owners of B(k,:), they solve, X(k,:) goes down each process column,
    the panel tiles A(:,k) are delivered (one batched p2p exchange) to the
    owners of the B rows they update, packed in local-row order, and ONE
    GEMM updates all of this rank's remaining rows."""
    sB = B.storage
    bcB = sB.bc
    comm = sB.comm
    grid = grid_of(B)
    lbB = B.local_block(slot)
    dev = lbB.data.device
    nb, p, q, pr, pc = bcB.nb, bcB.p, bcB.q, bcB.pr, bcB.pc
    lower = A.uploLogical() == Uplo.Lower
    diag = A.diag().value
    opA = A.op()
    upl = A.uploPhysical().value if hasattr(A.uploPhysical(), "value") else 'L'
    mt = B.mt()
    rB0, _ = B.global_offsets()
    if rB0 % nb:
        raise SlateError("trsm: B must start on a tile boundary")
    gb0 = rB0 // nb
    if alpha != 1 and lbB.mloc and lbB.nloc:
        ops.gescale(alpha, lbB.data)
    order = range(mt) if lower else range(mt - 1, -1, -1)
    sA = A.storage

    def stored_key(i, k):
        return A._global_ij(i, k)

    def owner(key):
        return sA.tileRank(key)

    def get_tile(key):
        return sA.tile_data(key[0], key[1], sA.origin_slot)

    def shape(key):
        return sA.tileMb(key[0]), sA.tileNb(key[1])

    procrow_ranks = {}
    for r in range(comm.size):
        procrow_ranks.setdefault(grid.coords(r)[0], []).append(r)
    for k in order:
        gk = gb0 + k
        kb = B.tileMb(k)
        rows = list(range(k + 1, mt)) if lower else list(range(0, k))
        needs = {}
        for rp in range(p):
            ks = [stored_key(k, k)] if (gk % p) == rp else []
            ks += [stored_key(i, k) for i in rows if ((gb0 + i) % p) == rp]
            for r in procrow_ranks.get(rp, []):
                needs[r] = ks
        got = exchange_tiles(comm, needs, owner, get_tile, shape, sB.dtype, dev)
        Xk = ops.colmajor_empty(kb, lbB.nloc, sB.dtype, dev)
        if (gk % p) == pr and lbB.nloc:
            lr = tiles_local_before(gk, p, pr) * nb - lbB.row_off
            Bk = lbB.data[lr:lr + kb, :]
            ops.trsm('L', upl, opA.value, diag, 1.0, got[stored_key(k, k)], Bk)
            Xk.copy_(Bk)
        if lbB.nloc and p > 1:
            grid.col_comm.bcast(Xk, gk % p)
        my_rows = [i for i in rows if ((gb0 + i) % p) == pr]
        if my_rows and lbB.nloc:
            # my updated rows are one contiguous local range of B
            lr0 = tiles_local_before(gb0 + my_rows[0], p, pr) * nb - lbB.row_off
            tot = sum(B.tileMb(i) for i in my_rows)
            Lm = ops.colmajor_empty(tot, kb, sB.dtype, dev)
            off = 0
            for i in my_rows:
                mi = B.tileMb(i)
                ops.gecopy(got[stored_key(i, k)], Lm[off:off + mi], trans=opA.value)
                off += mi
            ops.gemm(-1.0, Lm, Xk, 1.0, lbB.data[lr0:lr0 + tot, :])
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
