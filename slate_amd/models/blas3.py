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
from ..core.enums import Diag, MethodGemm, MethodHemm, MethodTrsm, Op, Option, Side, Uplo
from ..core.exceptions import SlateError
from ..core.options import get_option
from ..core.storage import DEV, l2g
from ..parallel.streams import StreamSet
from ..utils.trace import trace_block
from ._panels import assemble_cols, col_bcast, plan_col_gather, row_bcast
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
        if _hemm_method(B, opts) == MethodHemm.A:
            return _hemmA(side, alpha, A, B, beta, C, opts, _sym)
        return _hemmC(side, alpha, A, B, beta, C, opts, _sym)


def _hemm_method(B, opts):
    """src/hemm.cc:11-24: stationary A when B has a single block column."""
    m = get_option(opts, Option.MethodHemm, MethodHemm.Auto)
    if m in (MethodHemm.A, MethodHemm.C):
        return m
    return MethodHemm.A if B.nt() < 2 else MethodHemm.C


def _hemmC(side, alpha, A, B, beta, C, opts, sym):
    """Stationary-C hemm (src/hemmC.cc:147-429) without materialising the
    full Hermitian matrix: the Right side goes through the transposed Left
    problem, as _hemmA does."""
    slot = target_slot(C, opts)
    if side == Side.Right:
        cplx = C.storage.dtype.is_complex and not sym
        tr = (lambda X: X.conj_transpose()) if cplx else (lambda X: X.transpose())
        cj = (lambda v: complex(v).conjugate()) if cplx else (lambda v: v)
        Bt = _copy_in(tr(B), C, slot)
        Ct = _copy_in(tr(C), C, slot)
        _hemmC_left(cj(alpha), A, Bt, cj(beta), Ct, slot, sym)
        _copy_out(tr(Ct), C)
        return C
    Bw = B if (_at_origin(B) and _same_grid(B, C)) else _copy_in(B, C, slot)
    Cw = C if _at_origin(C) else _fresh(C, C.m(), C.n(), slot)
    if Cw is not C and beta != 0:
        _copy_out(C, Cw)
    _hemmC_left(alpha, A, Bw, beta, Cw, slot, sym)
    if Cw is not C:
        _copy_out(Cw, C)
    return C


# per-rank workspace of the last _hemmC_left call (tests): peak elements
HEMMC_STATS = {"workspace_elems": 0}


def _hemmC_left(alpha, A, B, beta, C, slot, sym):
    """Left hemmC, SUMMA over k with the block column k of the FULL matrix
    assembled per step from the stored triangle only (SLATE broadcasts the
    A(:, k) tiles and the transposed A(k, :) tiles of each step,
    src/hemmC.cc:147-429).  For stored Lower, block column k is A(i, k)
    (i >= k, stored, on process column k % q) over op(A(k, i)) (i < k, the
    stored block row k, op = ^H or ^T).  Per step:
      1. the block row k goes down each process column (one column
         broadcast of its mirror-range local columns);
      2. each rank writes into a zeroed (local rows x kb) buffer the tiles
         it can: the direct tiles when it is on process column k % q (the
         diagonal tile symmetrised from its stored triangle), and op() of
         the mirror tiles whose column lands on its own process column;
      3. ONE all-reduce over the row communicator completes the block column
         on every rank of the row (every tile is written by exactly one
         process column; x + 0 is exact);
      4. B(k, :) goes down the process columns and ONE GEMM updates the
         local C.
    Workspace per rank: (local rows + local cols) x nb -- never the n x n
    matrix the former full-copy redistribution built."""
    if not (_same_grid(A, C) and A.global_offsets() == (0, 0) and A.op() == Op.NoTrans
            and A.local_block(slot).mloc == C.local_block(slot).mloc):
        A = _copy_herm(A, C, slot)
    sC = C.storage
    bc = sC.bc
    grid = grid_of(C)
    lbA = A.local_block(slot)
    lbB = B.local_block(slot)
    lbC = C.local_block(slot)
    dev = lbC.data.device
    dt = sC.dtype
    nb, p, q, pr, pc = bc.nb, bc.p, bc.q, bc.pr, bc.pc
    n = A.n()
    mt = (n + nb - 1) // nb
    mloc, nlocA, nloc = lbA.mloc, lbA.nloc, lbC.nloc
    lower = A.uploPhysical() == Uplo.Lower
    up = 'L' if lower else 'U'
    other = 'U' if lower else 'L'
    op = 'T' if (sym or not dt.is_complex) else 'C'
    Aloc = lbA.data
    HEMMC_STATS["workspace_elems"] = 0
    for k in range(mt):
        kb = min(nb, n - k * nb)
        rk, ck = k % p, k % q
        lrk = tiles_local_before(k, p, pr) * nb
        lck = tiles_local_before(k, q, pc) * nb
        Acol = ops.colmajor_zeros(mloc, kb, dt, dev)
        # 2a. direct tiles (stored column block k)
        if pc == ck and mloc:
            d0, d1 = (tiles_local_before(k + 1, p, pr) * nb, mloc) if lower else (0, lrk)
            if d1 > d0:
                ops.gecopy(Aloc[d0:d1, lck:lck + kb], Acol[d0:d1])
            if pr == rk:
                Dk = Aloc[lrk:lrk + kb, lck:lck + kb]
                Ad = Acol[lrk:lrk + kb]
                ops.gecopy(Dk, Ad, uplo=up)
                ops.gecopy(Dk, Ad, uplo=other, trans=op)
                if op == 'C':
                    d = torch.diagonal(Ad)
                    d.copy_(d.real.to(dt))
        # 1. block row k (its mirror-range local columns) down the column
        m0, m1 = (0, lck) if lower else (tiles_local_before(k + 1, q, pc) * nb, nlocA)
        src = Aloc[lrk:lrk + kb, m0:m1] if pr == rk else None
        Rk = col_bcast(grid, src, rk, kb, m1 - m0, dt, dev) if m1 > m0 else None
        # 2b. mirror tiles i with i % p == pr and i % q == pc
        if Rk is not None:
            tiles = range(pr, k, p) if lower else range(k + 1 + ((pr - k - 1) % p), mt, p)
            for i in tiles:
                if i % q != pc:
                    continue
                wi = min(nb, n - i * nb)
                lri = tiles_local_before(i, p, pr) * nb
                lci = tiles_local_before(i, q, pc) * nb - m0
                ops.gecopy(Rk[:, lci:lci + wi], Acol[lri:lri + wi], trans=op)
        # 3. complete the block column along the process row
        if q > 1 and mloc:
            grid.row_comm.allreduce(Acol)
        # 4. B(k, :) down the process columns, one GEMM
        srcB = lbB.data[lrk:lrk + kb, :] if pr == rk else None
        Bp = col_bcast(grid, srcB, rk, kb, nloc, dt, dev)
        HEMMC_STATS["workspace_elems"] = max(HEMMC_STATS["workspace_elems"],
                                             Acol.numel() + (Rk.numel() if Rk is not None else 0)
                                             + (Bp.numel() if Bp is not None else 0))
        if mloc and nloc:
            ops.gemm(alpha, Acol, Bp, beta if k == 0 else 1.0, lbC.data)
    if mt == 0 and mloc and nloc:
        ops.gescale(beta, lbC.data)
    _done(C)
    return C


def _hemmA(side, alpha, A, B, beta, C, opts, sym):
    """Right side through the transposed Left problem: C = alpha B A + beta
    C  <=>  C^H = conj(alpha) A B^H + conj(beta) C^H  (A Hermitian; ^T and
    no conjugation for symmetric A)."""
    slot = target_slot(C, opts)
    if side == Side.Right:
        cplx = C.storage.dtype.is_complex and not sym
        tr = (lambda X: X.conj_transpose()) if cplx else (lambda X: X.transpose())
        cj = (lambda v: complex(v).conjugate()) if cplx else (lambda v: v)
        Bt = _copy_in(tr(B), C, slot)
        Ct = _copy_in(tr(C), C, slot)
        _hemmA_left(cj(alpha), A, Bt, cj(beta), Ct, slot, sym)
        _copy_out(tr(Ct), C)
        return C
    Bw = B if (_at_origin(B) and _same_grid(B, C)) else _copy_in(B, C, slot)
    Cw = C if _at_origin(C) else _fresh(C, C.m(), C.n(), slot)
    if Cw is not C and beta != 0:
        _copy_out(C, Cw)
    _hemmA_left(alpha, A, Bw, beta, Cw, slot, sym)
    if Cw is not C:
        _copy_out(Cw, C)
    return C


def _hemmA_left(alpha, A, B, beta, C, slot, sym):
    """Stationary-A hemm (src/hemmA.cc): only the stored triangle of A is
    read and A never moves.  With T = stored triangle (diagonal included)
    and S = strict stored triangle, A = T + S^H, so per block column jb of
    B:  P = T_loc B(my A cols, jb)  is a partial sum for my local C rows and
    Q = S_loc^H B(my A rows, jb)  one for the C rows of my local A columns.
    Q is summed down the process column, its rows that belong to my process
    row are added into P, and P is reduced along the process row onto the
    owner of C(:, jb) (tile reduce, the reference's listReduce)."""
    import numpy as np
    if not (_same_grid(A, C) and A.global_offsets() == (0, 0) and A.op() == Op.NoTrans
            and A.local_block(slot).mloc == C.local_block(slot).mloc):
        A = _copy_herm(A, C, slot)
    sC = C.storage
    bc = sC.bc
    grid = grid_of(C)
    lbA = A.local_block(slot)
    lbB = B.local_block(slot)
    lbC = C.local_block(slot)
    dev = lbC.data.device
    dt = sC.dtype
    nb, p, q, pr, pc = bc.nb, bc.p, bc.q, bc.pr, bc.pc
    n = A.n()
    mloc, nlocA = lbA.mloc, lbA.nloc
    lower = A.uploPhysical() == Uplo.Lower
    Aloc = lbA.data
    T = ops.colmajor_empty(mloc, nlocA, dt, dev)
    Sx = ops.colmajor_empty(mloc, nlocA, dt, dev)
    if mloc and nlocA:
        # stored triangle / strict stored triangle by the block-cyclic mask
        # kernel (one launch each)
        mode = 1 if lower else 2
        ops.gecopy_mask(Aloc, T, (mode, nb, p, pr, q, pc, 0, 0, 0), real_diag=dt.is_complex and not sym)
        ops.gecopy_mask(Aloc, Sx, (mode, nb, p, pr, q, pc, 0, 0, -1))
    # rows of Q (my local A column tiles k) that land in my process row:
    # local A column offset t*nb -> local C row offset of tile k (one
    # contiguous range per tile)
    ks = np.arange(pc, (n + nb - 1) // nb, q, dtype=np.int64)
    lens = np.minimum(nb, n - ks * nb)
    qoff = np.cumsum(lens) - lens
    mine = ks % p == pr
    moves = [(int(qo), tiles_local_before(int(k), p, pr) * nb, int(ln))
             for k, qo, ln in zip(ks[mine], qoff[mine], lens[mine])]
    plan = plan_col_gather(B.storage.tileMb, 0, A.nt(), nb, p, q, pc, dev)
    ct = 'T' if sym else conj_trans(dt)
    for jb in range(C.nt()):
        owner = jb % q
        wb = C.tileNb(jb)
        lcb = tiles_local_before(jb, q, pc) * nb - lbB.col_off
        src = lbB.data[:, lcb:lcb + wb] if pc == owner else None
        Prow = row_bcast(grid, src, owner, lbB.mloc, wb, dt, dev)
        Bq = assemble_cols(plan, Prow, grid, p, wb, dt, dev)
        P = ops.colmajor_zeros(mloc, wb, dt, dev)
        Q = ops.colmajor_zeros(nlocA, wb, dt, dev)
        if mloc and nlocA:
            ops.gemm(1.0, T, Bq, 0.0, P)
            ops.gemm(1.0, Sx, Prow, 0.0, Q, ct, 'N')
        if p > 1 and nlocA:
            grid.col_comm.allreduce(Q)
        for qo, lr, ln in moves:
            ops.geadd(1.0, Q[qo:qo + ln], 1.0, P[lr:lr + ln])
        if q > 1 and mloc:
            grid.row_comm.reduce(P, owner)
        if pc == owner and lbC.mloc:
            lcc = tiles_local_before(jb, q, pc) * nb - lbC.col_off
            Cj = lbC.data[:, lcc:lcc + wb]
            if beta == 0:                       # C is not read when beta = 0
                ops.gecopy(P, Cj)
                if alpha != 1:
                    ops.gescale(alpha, Cj)
            else:
                ops.geadd(alpha, P, beta, Cj)
    _done(C)
    return C


def _copy_herm(A, like, slot):
    """Stored triangle of a Hermitian/symmetric A on like's grid, at the
    storage origin."""
    from ..core.matrix import HermitianMatrix
    from ..parallel.redist import redistribute_pieces
    W = _fresh(like, A.n(), A.n(), slot, cls=HermitianMatrix, uplo=A.uploPhysical())
    Ab = A if A.op() == Op.NoTrans else (A.conj_transpose() if A.op() == Op.ConjTrans else A.transpose())
    redistribute_pieces(Ab, W, uplo=A.uploPhysical())
    return W


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
        return _tri_dist("mm", side, alpha, A, B, opts)


def trsm(side, alpha, A, B, opts=None):
    """Solve op(A) X = alpha B (Left) or X op(A) = alpha B (Right); B <- X.
    Option.MethodTrsm: B (stationary B, work::trsm), A (stationary A with
    partial-sum reduces, work::trsmA); Auto picks A when B has a single
    block column (src/trsm.cc:12-21)."""
    side = Side.from_string(side) if not isinstance(side, Side) else side
    with trace_block("trsm"):
        if _single(A, B) and B.op() == Op.NoTrans:
            a, ta, _ = _loc(A)
            b, _, _ = _loc(B)
            uplo, diag = _tri_args(A)
            ops.trsm(side.value, uplo, ta, diag, alpha, a, b)
            _done(B)
            return B
        return _tri_dist("sm", side, alpha, A, B, opts)


def _trsm_method(B, opts):
    m = get_option(opts, Option.MethodTrsm, MethodTrsm.Auto)
    if m in (MethodTrsm.A, MethodTrsm.B):
        return m
    return MethodTrsm.A if B.nt() < 2 else MethodTrsm.B


def _tri_dist(kind, side, alpha, A, B, opts):
    """Distributed trmm ("mm") / trsm ("sm").  Right side by the transposed
    Left problem: X op(A) = alpha B  <=>  op(A)^H X^H = conj(alpha) B^H
    (^T when op(A) = A^T), one transposing redistribution each way.  The
    Left problem runs on B's grid with B at its storage origin (a sub-view B
    is copied into a fresh matrix and back) and op(A) as a NoTrans
    triangle whose tile rows coincide with B's (_tri_work)."""
    slot = target_slot(B, opts)
    if side == Side.Right:
        use_h = A.op() != Op.Trans
        tr = (lambda X: X.conj_transpose()) if use_h else (lambda X: X.transpose())
        Bw = B if B.op() == Op.NoTrans else _copy_in(B, B, slot)
        Bt = _copy_in(tr(Bw), Bw, slot)
        a2 = complex(alpha).conjugate() if (use_h and B.storage.dtype.is_complex) else alpha
        _tri_left(kind, a2, tr(A), Bt, slot, opts)
        _copy_out(tr(Bt), B)
        return B
    if not _at_origin(B):
        Bw = _copy_in(B, B, slot)
        _tri_left(kind, alpha, A, Bw, slot, opts)
        _copy_out(Bw, B)
        return B
    return _tri_left(kind, alpha, A, B, slot, opts)


def _tri_work(A, B, slot):
    """op(A) as a NoTrans triangular matrix on B's grid, at its storage
    origin, so that its tile row i lives on the process row of B's tile row
    i: A itself when it already is, else ONE redistribution of the stored
    triangle (transposing / conjugating when op(A) != NoTrans)."""
    from ..core.matrix import TriangularMatrix
    ok = A.op() == Op.NoTrans and _same_grid(A, B) and A.global_offsets() == (0, 0) \
        and A.last_mb is None and A.last_nb is None and A.m() == B.m() \
        and A.local_block(slot).mloc == B.local_block(slot).mloc
    if ok:
        return A
    from ..parallel.redist import redistribute_pieces
    F = _fresh(B, A.m(), A.n(), slot)
    redistribute_pieces(A, F, uplo=A.uplo())
    return TriangularMatrix(A.uplo(), F, diag=A.diag())


def _tri_left(kind, alpha, A, B, slot, opts):
    A = _tri_work(A, B, slot)
    if kind == "sm" and _trsm_method(B, opts) == MethodTrsm.A:
        return _trsmA_left(alpha, A, B, slot)
    return _tri_left_panels(kind, alpha, A, B, slot, opts)


def _tri_left_panels(kind, alpha, A, B, slot, opts=None):
    """Stationary-B Left trmm / trsm (src/work/work_trmm.cc,
    src/work/work_trsm.cc:102-265) with A and B tile-row aligned.  Step k:
    the block column A(:, k) goes along each process row (one row
    broadcast of the local rows), the block row X(k, :) down each process
    column (one column broadcast), then ONE GEMM updates this rank's rows
    on the triangle's side of k -- the updates touch only the stored
    triangle, so trmm costs the triangular flop count (m^2 n), not a dense
    product.  trsm solves tile row k on its owners first (forward for
    Lower); trmm runs the other way (backward for Lower) so that X(k, :) is
    still the input row when it is read, and applies A(k, k) last."""
    sB = B.storage
    bc = sB.bc
    grid = grid_of(B)
    lbA = A.local_block(slot)
    lbB = B.local_block(slot)
    dev = lbB.data.device
    dt = sB.dtype
    nb, p, q, pr, pc = bc.nb, bc.p, bc.q, bc.pr, bc.pc
    mloc, nloc = lbB.mloc, lbB.nloc
    lower = A.uplo() == Uplo.Lower
    upl, diag = ('L' if lower else 'U'), A.diag().value
    solve = kind == "sm"
    mt = B.mt()
    if solve and alpha != 1 and mloc and nloc:
        ops.gescale(alpha, lbB.data)
    forward = lower if solve else not lower
    steps = list(range(mt) if forward else range(mt - 1, -1, -1))
    # lookahead (SLATE work_trsm's lookahead tasks, work_trsm.cc:102-265):
    # the A block column of step k + 1 .. k + la travels along the process
    # row on the panel stream (the row communicator's one stream) while the
    # solve / column broadcast / GEMM of step k run on the update stream (the
    # column communicator's) -- A never depends on B, so the prefetch is
    # always legal
    la = max(0, int(get_option(opts, Option.Lookahead, 1)))
    ss = StreamSet(dev, reserve_cus=0)
    ss.fork()
    us = ss.update[0]
    fetched = {}

    def fetch(i):
        k = steps[i]
        kb = B.tileMb(k)
        lc = tiles_local_before(k, q, pc) * nb - lbA.col_off
        with ss.use(ss.panel):
            src = lbA.data[:, lc:lc + kb] if k % q == pc else None
            P = row_bcast(grid, src, k % q, mloc, kb, dt, dev)
            fetched[i] = (P, ss.event(ss.panel))

    for i in range(min(la + 1, len(steps))):
        fetch(i)
    for i, k in enumerate(steps):
        Prow, ev = fetched.pop(i)
        kb = B.tileMb(k)
        lrk = tiles_local_before(k, p, pr) * nb
        own = k % p == pr
        r0, r1 = (tiles_local_before(k + 1, p, pr) * nb, mloc) if lower else (0, lrk)
        with ss.use(us):
            ss.wait(us, ev)
            if Prow is not None and Prow.is_cuda:
                Prow.record_stream(us)
            Bk = lbB.data[lrk:lrk + kb, :] if own else None
            if solve:
                if own and nloc:
                    ops.trsm('L', upl, 'N', diag, 1.0, Prow[lrk:lrk + kb], Bk)
                Xk = col_bcast(grid, Bk, k % p, kb, nloc, dt, dev)
                if r1 > r0 and nloc:
                    ops.gemm(-1.0, Prow[r0:r1], Xk, 1.0, lbB.data[r0:r1])
            else:
                Xk = col_bcast(grid, Bk, k % p, kb, nloc, dt, dev)
                if r1 > r0 and nloc:
                    ops.gemm(alpha, Prow[r0:r1], Xk, 1.0, lbB.data[r0:r1])
                if own and nloc:
                    ops.trmm('L', upl, 'N', diag, alpha, Prow[lrk:lrk + kb], Bk)
        if i + la + 1 < len(steps):
            fetch(i + la + 1)
    ss.join()
    _done(B)
    return B


def _local_globals(nloc, nb, p, pr, n):
    """Global indices of the nloc local rows of process row pr (numpy)."""
    import numpy as np
    from ._panels import _ranges
    tiles = np.arange(pr, (n + nb - 1) // nb, p, dtype=np.int64)
    lens = np.minimum(nb, n - tiles * nb)
    return _ranges(tiles * nb, lens)[:nloc]


def _trsmA_left(alpha, A, B, slot):
    """Stationary-A Left trsm (src/work/work_trsmA.cc): A never moves.  The
    update A(i, k) X(k) runs on the owner of A(i, k) and accumulates into a
    per-rank partial sum W of its local rows; before tile row k is solved,
    the partial sums of that row are reduced over the process row onto the
    owner of A(k, k) together with alpha B(k, :), which solves and
    broadcasts X(k, :) back along its process row (to B's owners) and down
    its process column (to the owners of A(:, k)).  Used when B is skinny
    (one block column), where stationary B would leave all but one process
    column idle."""
    sB = B.storage
    bc = sB.bc
    grid = grid_of(B)
    lbA = A.local_block(slot)
    lbB = B.local_block(slot)
    dev = lbB.data.device
    dt = sB.dtype
    nb, p, q, pr, pc = bc.nb, bc.p, bc.q, bc.pr, bc.pc
    mloc, nloc = lbB.mloc, lbB.nloc
    n = B.n()
    lower = A.uplo() == Uplo.Lower
    upl, diag = ('L' if lower else 'U'), A.diag().value
    mt = B.mt()
    # my local columns of B as (local offset, global offset, width) tile runs
    cruns = [(tiles_local_before(t, q, pc) * nb, t * nb, min(nb, n - t * nb))
             for t in range(pc, (n + nb - 1) // nb, q)]
    W = ops.colmajor_zeros(mloc, n, dt, dev)
    for k in (range(mt) if lower else range(mt - 1, -1, -1)):
        kb = B.tileMb(k)
        lrk = tiles_local_before(k, p, pr) * nb
        dq = k % q
        if k % p == pr:
            S = ops.colmajor_zeros(kb, n, dt, dev)
            for lo, go, wd in cruns:
                ops.gecopy(lbB.data[lrk:lrk + kb, lo:lo + wd], S[:, go:go + wd])
            # S = alpha B(k, :) - W(k, :)
            ops.geadd(-1.0, W[lrk:lrk + kb], alpha, S)
            if q > 1:
                grid.row_comm.reduce(S, dq)
            if pc == dq:
                lc = tiles_local_before(k, q, pc) * nb - lbA.col_off
                ops.trsm('L', upl, 'N', diag, 1.0, lbA.data[lrk:lrk + kb, lc:lc + kb], S)
            if q > 1:
                grid.row_comm.bcast(S, dq)
            for lo, go, wd in cruns:
                ops.gecopy(S[:, go:go + wd], lbB.data[lrk:lrk + kb, lo:lo + wd])
            Xk = S
        else:
            Xk = ops.colmajor_empty(kb, n, dt, dev) if pc == dq else None
        if pc == dq:
            if p > 1:
                grid.col_comm.bcast(Xk, k % p)
            r0, r1 = (tiles_local_before(k + 1, p, pr) * nb, mloc) if lower else (0, lrk)
            if r1 > r0:
                lc = tiles_local_before(k, q, pc) * nb - lbA.col_off
                ops.gemm(1.0, lbA.data[r0:r1, lc:lc + kb], Xk, 1.0, W[r0:r1])
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
