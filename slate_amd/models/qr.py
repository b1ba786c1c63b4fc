"""QR / LQ family: geqrf, unmqr, gelqf, unmlq, cholqr, gels (QR, LQ and
CholeskyQR least squares).

Reference: `src/geqrf.cc:22-272` (host panel `internal::geqrf` + TSQR
reduction tree `internal::ttqrt`, `internal::unmqr`/`ttmqr` trailing
updates, lookahead DAG), `src/unmqr.cc`, `src/gelqf.cc`, `src/unmlq.cc`,
`src/cholqr.cc`, `src/gels.cc`, `src/gels_qr.cc`, `src/gels_cholqr.cc`.

MI355X design:
* the panel is factored ON THE GPU by a recursive Householder QR whose
  combine steps are MFMA GEMM/TRMM (csrc/hip/geqrf.hip); it returns the
  compact-WY T of the whole panel and an explicit unit-lower V, so the
  trailing update is three GEMM-class calls  C -= V (T^H (V^H C));
* one process row (p == 1, incl. a single GPU): lookahead pipeline like
  potrf/getrf -- panel + lookahead columns on the high-priority stream, the
  bulk update on the low-priority stream;
* p > 1: instead of SLATE's per-tile TSQR tree, the panel column (m-k*nb
  rows x nb, at most a few hundred MB even at m = 2^17) is all-gathered
  inside the process column and factored redundantly by every rank of that
  column (deterministic kernels => bit-identical V, T, R), so no broadcast of
  the result is needed inside the column; V and T then go along the process
  row, and the update's V^H C is one all-reduce over the process column.
* LQ is the conjugate transpose of QR: gelqf factors A^H (kept in the
  factor object) and unmlq applies Q^H of it.

Factors: ``TriangularFactors`` holds, per panel k, the kb x kb T and tau
(replicated on every rank); the reflectors stay in A below the diagonal
exactly as in LAPACK/SLATE.
"""
from __future__ import annotations

import torch

from .. import ops
from ..core.enums import Diag, Op, Option, Side, Uplo
from ..core.exceptions import SlateError
from ..core.matrix import Matrix, TriangularFactors, TriangularMatrix
from ..core.options import get_option
from ..core.storage import l2g
from ..parallel.streams import StreamSet
from ..utils.trace import trace_block
from ._util import conj_trans, grid_of, target_slot, tiles_local_before


# ------------------------------------------------------------------ helpers
def _apply_qh(V, Tk, C, conj=True):
    """C -= V op(T) (V^H C), op = ^H (apply Q^H) or none (apply Q)."""
    if C.shape[1] == 0 or C.shape[0] == 0:
        return
    ct = conj_trans(C.dtype)
    kb = Tk.shape[0]
    W = ops.colmajor_empty(kb, C.shape[1], C.dtype, C.device)
    ops.gemm(1.0, V, C, 0.0, W, transA=ct)
    ops.trmm('L', 'U', ct if conj else 'N', 'N', 1.0, Tk, W)
    ops.gemm(-1.0, V, W, 1.0, C)


def _apply_qh_dist(Vloc, Tk, Cloc, col_comm, conj=True):
    """Distributed C -= V op(T) V^H C where rows of V and C are split over the
    process column: W = sum_r V_r^H C_r is one all-reduce."""
    ct = conj_trans(Cloc.dtype)
    kb = Tk.shape[0]
    nc = Cloc.shape[1]
    if nc == 0:
        return
    W = ops.colmajor_zeros(kb, nc, Cloc.dtype, Cloc.device)
    if Vloc.shape[0]:
        ops.gemm(1.0, Vloc, Cloc, 0.0, W, transA=ct)
    if col_comm is not None and col_comm.size > 1:
        Wt = W.t().contiguous()
        col_comm.allreduce(Wt)
        W = Wt.t()
    ops.trmm('L', 'U', ct if conj else 'N', 'N', 1.0, Tk, W)
    if Vloc.shape[0]:
        ops.gemm(-1.0, Vloc, W, 1.0, Cloc)


def _check(A):
    if A.op() != Op.NoTrans or A.ioffset or A.joffset or A.row0_offset or A.col0_offset:
        raise SlateError("geqrf: pass a whole (non-transposed) block-cyclic matrix")


# ------------------------------------------------------------------ geqrf
def geqrf(A, T: TriangularFactors, opts=None) -> int:
    """A = Q R.  R overwrites the upper triangle, reflectors the lower part;
    T receives the per-panel block-reflector factors."""
    s = A.storage
    if s.bc is None:
        from .aux import run_on_block_cyclic
        return run_on_block_cyclic(A, lambda B, o: geqrf(B, T, o), opts)
    _check(A)
    with trace_block("geqrf"):
        bc = s.bc
        if bc.mb != bc.nb:
            raise SlateError("geqrf: square tiles required")
        slot = target_slot(A, opts)
        buf = s.prepare_local(slot)
        la = max(0, int(get_option(opts, Option.Lookahead, 1)))
        T.clear()
        T.nb = bc.nb
        T.kind = "qr"
        if bc.p == 1:
            _geqrf_p1(A, buf, T, la)
        else:
            _geqrf_general(A, buf, T)
        s.mark_local_modified(slot)
    return 0


def _geqrf_p1(A, buf, T, la):
    s = A.storage
    bc = s.bc
    nb, q, pc = bc.nb, bc.q, bc.pc
    m, n = s.m, s.n
    kt = min(s.mt, s.nt)
    dev, dt = buf.device, s.dtype
    grid = grid_of(A) if q > 1 else None
    nloc = bc.nloc
    ss = StreamSet(dev, reserve_cus=0)   # GEMM-shaped CholeskyQR panel: no reserved CUs (measured 32.5 vs 29.8 TF/s with 64)
    ev_tr = {}
    ss.fork()
    for k in range(kt):
        r0 = k * nb
        kb = min(nb, n - r0, m - r0)
        mk = m - r0
        own = (k % q) == pc
        lck = tiles_local_before(k, q, pc) * nb
        lc1 = min(tiles_local_before(k + 1, q, pc) * nb, nloc)
        lcla = min(tiles_local_before(k + 1 + la, q, pc) * nb, nloc)
        with ss.use(ss.panel):
            tau = torch.zeros(kb, dtype=dt, device=dev)     # on the panel stream
            if k - la - 1 >= 0:
                ss.wait(ss.panel, ev_tr[k - la - 1])
            with trace_block("geqrf::panel"):
                Tk = ops.colmajor_empty(kb, kb, dt, dev)
                V = ops.colmajor_empty(mk, kb, dt, dev)
                if own:
                    ops.geqrf(buf[r0:m, lck:lck + kb], tau, Tk, V)
                if q > 1:
                    from ..parallel.tilecomm import bcast_tile
                    bcast_tile(grid.row_comm, V, k % q)
                    bcast_tile(grid.row_comm, Tk, k % q)
                    grid.row_comm.bcast(tau, k % q)
            # newest lookahead column k+la: first part of step k-1's trailing
            if k >= 1 and la > 0:
                ss.wait(ss.panel, ev_tr[k - 1])
            if lcla > lc1:
                _apply_qh(V, Tk, buf[r0:m, lc1:lcla])
            ev_panel = ss.event(ss.panel)
        T.append({"T": Tk, "tau": tau, "r0": r0, "kb": kb})
        us = ss.update[0]
        with ss.use(us):
            ss.wait(us, ev_panel)
            if nloc > lcla and V.is_cuda:
                V.record_stream(us)
                Tk.record_stream(us)
            lcnx = max(min(tiles_local_before(k + 2 + la, q, pc) * nb, nloc), lcla)
            with trace_block("geqrf::trailing"):
                if lcnx > lcla:
                    _apply_qh(V, Tk, buf[r0:m, lcla:lcnx])
                ev_tr[k] = ss.event(us)
                if nloc > lcnx:
                    _apply_qh(V, Tk, buf[r0:m, lcnx:nloc])
    ss.join()


def _gather_panel(buf, mloc, k, nb, m, p, pr, lc, kb, grid, dt, dev):
    """All-gather rows [k*nb, m) of local columns [lc, lc+kb) within the
    process column; returns (P in global row order, my-rows index)."""
    from ..core.storage import numroc
    r0 = k * nb
    lr_k = tiles_local_before(k, p, pr) * nb
    sizes = [max(0, numroc(m, nb, r, p) - tiles_local_before(k, p, r) * nb) for r in range(p)]
    mx = max(sizes) if sizes else 0
    pad = ops.colmajor_zeros(max(mx, 1), kb, dt, dev)
    mine = buf[lr_k:mloc, lc:lc + kb] if mloc > lr_k else buf[0:0, lc:lc + kb]
    if mine.shape[0]:
        pad[:mine.shape[0]].copy_(mine)
    allp = grid.col_comm.allgather(pad.t().contiguous())
    P = ops.colmajor_empty(m - r0, kb, dt, dev)
    idx = {}
    for r in range(p):
        lr = tiles_local_before(k, p, r) * nb
        gi = [l2g(lr + i, nb, r, p) - r0 for i in range(sizes[r])]
        idx[r] = torch.as_tensor(gi, dtype=torch.int64, device=dev)
        if sizes[r]:
            ops.row_scatter(allp[r][:, :sizes[r]].t(), P, idx[r])
    return P, idx[pr], mine


def _geqrf_general(A, buf, T):
    s = A.storage
    bc = s.bc
    grid = grid_of(A)
    nb, p, q, pr, pc = bc.nb, bc.p, bc.q, bc.pr, bc.pc
    m, n = s.m, s.n
    kt = min(s.mt, s.nt)
    dev, dt = buf.device, s.dtype
    mloc, nloc = bc.mloc, bc.nloc
    for k in range(kt):
        r0 = k * nb
        kb = min(nb, n - r0, m - r0)
        ck = k % q
        lr_k = tiles_local_before(k, p, pr) * nb
        lc_k = tiles_local_before(k, q, pc) * nb
        lc1 = min(tiles_local_before(k + 1, q, pc) * nb, nloc)
        tau = torch.zeros(kb, dtype=dt, device=dev)
        Tk = ops.colmajor_empty(kb, kb, dt, dev)
        nmine = max(0, mloc - lr_k)
        Vloc = ops.colmajor_empty(nmine, kb, dt, dev)
        with trace_block("geqrf::panel"):
            if pc == ck:
                P, myidx, mine = _gather_panel(buf, mloc, k, nb, m, p, pr, lc_k, kb, grid, dt, dev)
                V = ops.colmajor_empty(m - r0, kb, dt, dev)
                ops.geqrf(P, tau, Tk, V)            # redundant in the column: identical results
                if nmine:
                    ops.row_gather(P, mine, myidx)
                    ops.row_gather(V, Vloc, myidx)
        if q > 1:
            from ..parallel.tilecomm import bcast_tile
            bcast_tile(grid.row_comm, Vloc, ck)
            bcast_tile(grid.row_comm, Tk, ck)
            grid.row_comm.bcast(tau, ck)
        T.append({"T": Tk, "tau": tau, "r0": r0, "kb": kb})
        with trace_block("geqrf::trailing"):
            _apply_qh_dist(Vloc, Tk, buf[lr_k:mloc, lc1:nloc], grid.col_comm)


# ------------------------------------------------------------------ unmqr
def _same_rows(A, C):
    a, c = A.storage.bc, C.storage.bc
    return (a.mb, a.p, a.pr) == (c.mb, c.p, c.pr) and C.global_offsets()[0] == 0 and \
        a.order == c.order and A.storage.comm is C.storage.comm
def _local_V(A, k, Tk):
    """Explicit V rows of panel k for this rank's local rows >= k*nb,
    available on every rank of the process row (bcast along the row)."""
    s = A.storage
    bc = s.bc
    nb, p, q, pr, pc = bc.nb, bc.p, bc.q, bc.pr, bc.pc
    kb = Tk["kb"]
    lr_k = tiles_local_before(k, p, pr) * nb
    lc_k = tiles_local_before(k, q, pc) * nb
    mloc = bc.mloc
    buf = s.local[s.origin_slot]
    nmine = max(0, mloc - lr_k)
    Vloc = ops.colmajor_empty(nmine, kb, s.dtype, buf.device)
    if pc == k % q and nmine:
        # rows of the global diagonal block need the unit-lower structure
        src = buf[lr_k:mloc, lc_k:lc_k + kb]
        if pr == k % p:
            ops.v_explicit(src, Vloc)     # my first local rows ARE the diagonal block
        else:
            Vloc.copy_(src)
    if q > 1:
        from ..parallel.tilecomm import bcast_tile
        bcast_tile(grid_of(A).row_comm, Vloc, k % q)
    return Vloc, lr_k


def unmqr(side, op, A, T: TriangularFactors, C, opts=None):
    """C = op(Q) C (Left) or C op(Q) (Right), Q from geqrf(A, T)."""
    with trace_block("unmqr"):
        sA, sC = A.storage, C.storage
        if sA.bc is None or sC.bc is None:
            raise SlateError("unmqr: block-cyclic A and C required")
        if C.op() != Op.NoTrans:
            raise SlateError("unmqr: C must not be transposed")
        conj = op != Op.NoTrans
        kt = len(T)
        if side == Side.Left and not _same_rows(A, C):
            Cc = _new_like(A, C.m(), C.n())
            from .aux import copy
            copy(C, Cc)
            unmqr(side, op, A, T, Cc, opts)
            copy(Cc, C)
            return 0
        if side == Side.Left:
            order = range(kt) if conj else range(kt - 1, -1, -1)
            lbC = C.local_block()
            cbuf = lbC.data
            grid = grid_of(C)
            for k in order:
                Vloc, lr_k = _local_V(A, k, T[k])
                Cl = cbuf[lr_k - lbC.row_off:, :] if lr_k >= lbC.row_off else cbuf
                _apply_qh_dist(Vloc, T[k]["T"], Cl, grid.col_comm, conj=conj)
        else:
            # C op(Q) = (op(Q)^H C^H)^H: work on the conjugate transpose
            from .aux import copy_conj_transpose
            Ch = _conj_transposed_copy(C, A)
            unmqr(Side.Left, Op.NoTrans if conj else Op.ConjTrans, A, T, Ch, opts)
            copy_conj_transpose(Ch, C)
        sC.mark_local_modified(sC.origin_slot)
    return 0


# ------------------------------------------------------------------ LQ
def gelqf(A, T: TriangularFactors, opts=None) -> int:
    """A = L Q: computed as the QR of A^H (kept in T.At); L and the row
    reflectors are written back into A in LAPACK layout."""
    from .aux import copy_conj_transpose
    with trace_block("gelqf"):
        At = _conj_transposed_copy(A, A)
        geqrf(At, T, opts)
        T.kind = "lq"
        T.At = At
        copy_conj_transpose(At, A)
    return 0


def unmlq(side, op, A, T: TriangularFactors, C, opts=None):
    """C = op(Q) C or C op(Q) with Q from gelqf (Q_lq = Q_qr(A^H)^H)."""
    if getattr(T, "At", None) is None:
        raise SlateError("unmlq: factors from gelqf required")
    flip = Op.NoTrans if op != Op.NoTrans else Op.ConjTrans
    return unmqr(side, flip, T.At, T, C, opts)


# ------------------------------------------------------------------ CholQR
def cholqr(A, R, opts=None) -> int:
    """Cholesky QR (src/cholqr.cc): R^H R = A^H A (herk + potrf), Q = A R^{-1}
    overwrites A.  R is an n x n matrix (upper triangle filled)."""
    from .blas3 import herk, trsm
    from .chol import potrf
    from .aux import set as aset
    with trace_block("cholqr"):
        aset(0.0, 0.0, R)
        Rh = _hermitian_upper(R)
        herk(1.0, A.conj_transpose(), 0.0, Rh, opts)
        info = potrf(Rh, opts)
        if info:
            return info
        Rt = TriangularMatrix(Uplo.Upper, R, diag=Diag.NonUnit)
        trsm(Side.Right, 1.0, Rt, A, opts)
    return 0


def _hermitian_upper(R):
    from ..core.matrix import HermitianMatrix
    return HermitianMatrix(Uplo.Upper, R)


# ------------------------------------------------------------------ gels
def gels(A, T: TriangularFactors, BX, opts=None) -> int:
    """Least squares / minimum norm: min ||op(A) X - B||.  BX is
    max(m,n) x nrhs; on return its top rows hold X.  Method from
    Option.MethodGels ("qr" default, "cholqr")."""
    from .blas3 import trsm
    from ..core.enums import MethodGels
    method = get_option(opts, Option.MethodGels, MethodGels.QR)
    method = "cholqr" if method in (MethodGels.CholQR, "cholqr", "CholQR") else "qr"
    m, n = A.m(), A.n()
    nrhs = BX.n()
    with trace_block("gels"):
        if A.op() != Op.NoTrans:
            # op(A) = A^H: solve via the LQ/QR of the stored matrix
            from .aux import redistribute
            Ah = _new_like(A, m, n)      # materialise op(A) in NoTrans layout
            redistribute(A, Ah)
            return gels(Ah, T, BX, opts)
        if m >= n:
            if method == "cholqr":
                R = _new_like(A, n, n)
                info = cholqr(A, R, opts)
                if info:
                    return info
                # X = R^{-1} Q^H B   (Q = A now)
                B = BX.sub(0, BX.mt() - 1, 0, BX.nt() - 1)
                Y = _new_like(A, n, nrhs)
                from .blas3 import gemm
                gemm(1.0, A.conj_transpose(), B, 0.0, Y, opts)
                trsm(Side.Left, 1.0, TriangularMatrix(Uplo.Upper, R, diag=Diag.NonUnit), Y, opts)
                from .aux import copy
                Xtop = BX.slice(0, n - 1, 0, nrhs - 1)
                copy(Y, Xtop)
                return 0
            geqrf(A, T, opts)
            unmqr(Side.Left, Op.ConjTrans, A, T, BX, opts)
            R = TriangularMatrix(Uplo.Upper, A.slice(0, n - 1, 0, n - 1), diag=Diag.NonUnit)
            Xtop = BX.slice(0, n - 1, 0, nrhs - 1)
            trsm(Side.Left, 1.0, R, Xtop, opts)
        else:
            # minimum norm: A = L Q;  L Y = B (m rows);  X = Q^H [Y; 0]
            gelqf(A, T, opts)
            L = TriangularMatrix(Uplo.Lower, A.slice(0, m - 1, 0, m - 1), diag=Diag.NonUnit)
            Ytop = BX.slice(0, m - 1, 0, nrhs - 1)
            trsm(Side.Left, 1.0, L, Ytop, opts)
            from .aux import set as aset
            if n > m:
                aset(0.0, 0.0, BX.slice(m, n - 1, 0, nrhs - 1))
            unmlq(Side.Left, Op.ConjTrans, A, T, BX, opts)
    return 0


def gels_qr(A, T, BX, opts=None):
    return gels(A, T, BX, opts)


def gels_cholqr(A, BX, opts=None):
    o = dict(opts or {})
    from ..core.enums import MethodGels
    o[Option.MethodGels] = MethodGels.CholQR
    return gels(A, TriangularFactors(), BX, o)


def _dev_index(A):
    d = A.storage.device
    return d.index if d.type == "cuda" else -1


def _new_like(A, m, n):
    """New m x n matrix on A's process grid / tile size / device."""
    bc = A.storage.bc
    M = Matrix(m, n, nb=bc.nb, mb=bc.mb, p=bc.p, q=bc.q, comm=A.storage.comm, dtype=A.storage.dtype,
               device=A.storage.device, order=bc.order)
    M.insertLocalTiles(device=_dev_index(A))
    return M


def _conj_transposed_copy(A, like):
    """A^H as a new matrix distributed like `like` (dense all-gather path)."""
    from .aux import copy_conj_transpose
    B = _new_like(like, A.n(), A.m())
    copy_conj_transpose(A, B)
    return B
