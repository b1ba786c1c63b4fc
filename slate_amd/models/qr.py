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
* p > 1: TSQR over the process column (SLATE: internal::geqrf per tile +
  the ttqrt reduction tree, src/geqrf.cc:161-251).  Each rank of the panel's
  process column QR-factors ITS OWN panel rows on its GPU (O(m/p nb^2)), the
  kr x nb R factors are all-gathered (one collective of p nb^2 words) and
  every rank of the column factors the stacked [R_rk; R_rk+1; ...] redundantly
  (deterministic kernels => identical R^, V^, T^, so no broadcast inside the
  column); R^ lands in the diagonal tile.  The flat p-way stack replaces
  SLATE's binary tree: on a fully connected xGMI node one all-gather is one
  hop.  Local V_r, T_r and the tree's V^_r, T^ go along the process row in
  ONE packed broadcast; the trailing update is local (C_r -= V_r T_r^H V_r^H
  C_r) plus the tree part on the top rows, whose V^H C is one all-reduce over
  the column.  Lookahead as for p == 1, the update stream with its own
  column communicator.
* LQ is the conjugate transpose of QR: gelqf factors A^H (kept in the
  factor object) and unmlq applies Q^H of it.

Factors: ``TriangularFactors`` holds, per panel k, the kb x kb T and tau
(replicated on every rank); the reflectors stay in A below the diagonal
exactly as in LAPACK/SLATE.
"""
from __future__ import annotations

import os

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
from ..utils import watchdog as _wd


# ------------------------------------------------------------------ helpers
def _apply_qh(V, Tk, C, conj=True, Vh=None):
    """C -= V op(T) (V^H C), op = ^H (apply Q^H) or none (apply Q).  Vh:
    optional explicit V^H (kb x m), making V^H C an NN GEMM."""
    if C.shape[1] == 0 or C.shape[0] == 0:
        return
    ct = conj_trans(C.dtype)
    kb = Tk.shape[0]
    W = ops.colmajor_empty(kb, C.shape[1], C.dtype, C.device)
    if Vh is not None:
        ops.gemm(1.0, Vh, C, 0.0, W)
    else:
        ops.gemm(1.0, V, C, 0.0, W, transA=ct)
    ops.trmm('L', 'U', ct if conj else 'N', 'N', 1.0, Tk, W)
    ops.gemm(-1.0, V, W, 1.0, C)


def _vh(V):
    """Explicit V^H (kb x m) of a tall device reflector block, or None: with
    it the V^H C GEMM of _apply_qh runs as NN (see _geqrf_p1)."""
    if not V.is_cuda or V.shape[0] < _VH_MIN_ROWS or V.shape[1] == 0:
        return None
    Vh = ops.colmajor_empty(V.shape[1], V.shape[0], V.dtype, V.device)
    ops.gecopy(V, Vh, trans=conj_trans(V.dtype))
    return Vh


def _check(A):
    if A.op() != Op.NoTrans or A.ioffset or A.joffset or A.row0_offset or A.col0_offset:
        raise SlateError("geqrf: pass a whole (non-transposed) block-cyclic matrix")


# ------------------------------------------------------------------ geqrf
def geqrf(A, T: TriangularFactors, opts=None) -> int:
    """A = Q R.  R overwrites the upper triangle, reflectors the lower part;
    T receives the per-panel block-reflector factors.

    Memory: a host-origin matrix larger than the device budget is factored
    OUT OF CORE (left-looking block-column streaming) on ONE rank only.  On a
    p x q grid with p q > 1 every rank stages its whole local block on its
    GPU (288 GB of HBM3E per MI355X: a 2 x 4 grid holds n ~ 160k fp64 in
    core); a larger problem needs a larger grid (SLATE's workspace streaming
    for p x q, BaseMatrix.hh:2640-2781, is not implemented)."""
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
        la = max(0, int(get_option(opts, Option.Lookahead, 1)))
        T.clear()
        T.nb = bc.nb
        T.kind = "qr"
        if _maybe_ooc(A, s, slot, T, la):
            return 0
        buf = s.prepare_local(slot)
        if bc.p == 1:
            _geqrf_p1(A, buf, T, la)
        else:
            _geqrf_general(A, buf, T, la)
        s.mark_local_modified(slot)
    return 0


def _maybe_ooc(A, s, slot, T, la):
    """Host-origin matrix on one rank, larger than the device budget (or
    SLATE_AMD_OOC_COLS set): the left-looking out-of-core QR streams block
    columns (models/ooc.py).  True when it ran."""
    from .ooc import geqrf_ooc, ooc_applicable, ooc_block_columns
    if not ooc_applicable(A, s, slot):
        return False
    from ..core.storage import HOST
    dev = torch.device("cuda", torch.cuda.current_device())
    W = ooc_block_columns(s.m, s.n, s.bc.nb, s.dtype, dev, 5)
    if not W or W >= s.n:
        return False
    s.sync_origin()
    T.extend(geqrf_ooc(s.local[HOST][:s.m, :s.n], s.m, s.n, s.bc.nb, W, dev, la))
    s.mark_local_modified(HOST)
    return True


# panels at least this tall get an explicit V^H (SLATE_AMD_QR_VH_ROWS; 0 = never)
_VH_MIN_ROWS = int(os.environ.get("SLATE_AMD_QR_VH_ROWS", "4096")) or (1 << 62)


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
    # grouped bulk updates (SLATE_AMD_QR_GROUP=2, one process column; off by
    # default: dgeqrf 65536 x 8192 on one MI355X 38.3 vs 38.9 TF/s): the
    # bulk trailing columns of an even step wait one step and then take the
    # two panels as ONE block reflector (K = 2 nb: half the passes over the
    # trailing matrix, twice the GEMM depth); the lookahead columns and the
    # next step's newest lookahead column are updated per panel as before
    group = int(os.environ.get("SLATE_AMD_QR_GROUP", "1")) if q == 1 else 1
    pending = None
    ss.fork()
    for k in range(kt):
        _wd.beat(f"geqrf step {k}")
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
                # explicit V^H (one LDS-tiled transpose per step): the
                # V^H C GEMMs of this step run as NN instead of TN
                Vh = None
                if V.is_cuda and mk >= _VH_MIN_ROWS and nloc > lc1:
                    Vh = ops.colmajor_empty(kb, mk, dt, dev)
                    ops.gecopy(V, Vh, trans=conj_trans(dt))
            # newest lookahead column k+la: first part of step k-1's trailing
            if k >= 1 and la > 0:
                ss.wait(ss.panel, ev_tr[k - 1])
            if own and lck + kb < lc1:
                # wide matrix, last panel: fewer rows than the tile has
                # columns -- the tile's remaining columns are trailing too
                _apply_qh(V, Tk, buf[r0:m, lck + kb:lc1], Vh=Vh)
            if lcla > lc1:
                _apply_qh(V, Tk, buf[r0:m, lc1:lcla], Vh=Vh)
            ev_panel = ss.event(ss.panel)
        T.append({"T": Tk, "tau": tau, "r0": r0, "kb": kb, "kr": kb, "tree": None})
        us = ss.update[0]
        with ss.use(us):
            ss.wait(us, ev_panel)
            if nloc > lcla and V.is_cuda:
                V.record_stream(us)
                Tk.record_stream(us)
                if Vh is not None:
                    Vh.record_stream(us)
            lcnx = max(min(tiles_local_before(k + 2 + la, q, pc) * nb, nloc), lcla)
            with trace_block("geqrf::trailing"):
                if pending is not None:
                    # columns [lcla, nloc) still lack the previous panel:
                    # apply both panels as one block reflector
                    from .eig import _merge_reflectors
                    pr0, pV, pT = pending
                    g0, Vg, Tg = _merge_reflectors([(pr0, pV, pT), (r0, V, Tk)])
                    Vgh = _vh(Vg)
                    if lcnx > lcla:
                        _apply_qh(Vg, Tg, buf[g0:m, lcla:lcnx], Vh=Vgh)
                    ev_tr[k] = ss.event(us)
                    if nloc > lcnx:
                        _apply_qh(Vg, Tg, buf[g0:m, lcnx:nloc], Vh=Vgh)
                    pending = None
                else:
                    if lcnx > lcla:
                        _apply_qh(V, Tk, buf[r0:m, lcla:lcnx], Vh=Vh)
                    ev_tr[k] = ss.event(us)
                    if nloc > lcnx:
                        if group > 1 and k + 1 < kt and kb == nb and m - r0 > nb:
                            pending = (r0, V, Tk)          # the bulk waits for the next panel
                        else:
                            _apply_qh(V, Tk, buf[r0:m, lcnx:nloc], Vh=Vh)
    if pending is not None:
        raise SlateError("geqrf: grouped update left pending")
    ss.join()


def _pack(parts, dev):
    from .lu import _Pack
    return _Pack(parts, dev)


def _geqrf_general(A, buf, T, la):
    """p > 1 process rows: TSQR panel + lookahead (see module docstring)."""
    from ..core.storage import numroc
    s = A.storage
    bc = s.bc
    grid = grid_of(A)
    nb, p, q, pr, pc = bc.nb, bc.p, bc.q, bc.pr, bc.pc
    m, n = s.m, s.n
    kt = min(s.mt, s.nt)
    dev, dt = buf.device, s.dtype
    mloc, nloc = bc.mloc, bc.nloc
    nloc_r = [numroc(m, nb, r, p) for r in range(p)]
    ss = StreamSet(dev, reserve_cus=0)
    colc, rowc = grid.col_comm, grid.row_comm
    colu = grid.col_comm_u
    ev_tr = {}
    ss.fork()
    for k in range(kt):
        _wd.beat(f"geqrf step {k}")
        r0 = k * nb
        kb = min(nb, n - r0, m - r0)
        rk, ck = k % p, k % q
        lr_k = min(tiles_local_before(k, p, pr) * nb, mloc)
        lc_k = min(tiles_local_before(k, q, pc) * nb, nloc)
        lc1 = min(tiles_local_before(k + 1, q, pc) * nb, nloc)
        lcla = min(tiles_local_before(k + 1 + la, q, pc) * nb, nloc)
        lcnx = max(min(tiles_local_before(k + 2 + la, q, pc) * nb, nloc), lcla)
        cnt = [max(0, nloc_r[r] - min(tiles_local_before(k, p, r) * nb, nloc_r[r])) for r in range(p)]
        kr = [min(c, kb) for c in cnt]                   # local reflectors = stacked rows per rank
        order = [(rk + i) % p for i in range(p)]         # rk first: its top rows receive R^
        soff, o = {}, 0
        for r in order:
            soff[r] = o
            o += kr[r]
        tot = o
        ks = min(tot, kb)
        tree = sum(1 for r in range(p) if kr[r]) > 1
        nmine, km = cnt[pr], kr[pr]
        st = dict(k=k, kb=kb, rk=rk, lr_k=lr_k, lc_k=lc_k, nmine=nmine, km=km, kr=kr, soff=soff,
                  order=order, tot=tot, ks=ks, tree=tree)
        with ss.use(ss.panel):
            if k - la - 1 >= 0:
                ss.wait(ss.panel, ev_tr[k - la - 1])
            # small factors first (kept in T), the local V (re-derived from A
            # by unmqr) last
            parts = [("T", km, km, dt), ("tau", km, 1, dt)]
            if tree:
                parts += [("Vh", km, ks, dt), ("Th", ks, ks, dt), ("tauh", ks, 1, dt)]
            parts += [("V", nmine, km, dt)]
            pk = _pack(parts, dev)
            with trace_block("geqrf::panel"):
                if pc == ck:
                    _tsqr_panel(buf, mloc, pr, p, colc, pk, st, dt, dev)
                if q > 1:
                    rowc.bcast(pk.raw, ck)
            kp = pk.prefix("V")
            f = {"T": kp.get("T"), "tau": kp.get("tau")[:, 0], "r0": r0, "kb": kb, "kr": km,
                 "tree": ({"V": kp.get("Vh"), "T": kp.get("Th"), "tau": kp.get("tauh")[:, 0], "ks": ks}
                          if tree else None)}
            Vloc = pk.get("V")
            Vh = None
            if Vloc.is_cuda and nmine >= _VH_MIN_ROWS and km and nloc > lc1:
                Vh = ops.colmajor_empty(km, nmine, dt, dev)       # NN V^H C (see _geqrf_p1)
                ops.gecopy(Vloc, Vh, trans=conj_trans(dt))
            if k >= 1 and la > 0:
                ss.wait(ss.panel, ev_tr[k - 1])
            # (wide matrix, last panel: the tile's columns beyond kb are trailing too)
            part = [(lc_k + kb, lc1)] if (pc == ck and lc_k + kb < lc1) else []
            _tsqr_update(buf, lr_k, mloc, Vloc, f, part + [(lc1, lcla)], colc, dt, dev, Vh=Vh)
            ev_panel = ss.event(ss.panel)
        T.append(f)
        us = ss.update[0]
        with ss.use(us):
            ss.wait(us, ev_panel)
            if buf.is_cuda:
                pk.raw.record_stream(us)
                if Vh is not None:
                    Vh.record_stream(us)
            with trace_block("geqrf::trailing"):
                _tsqr_update(buf, lr_k, mloc, Vloc, f, [(lcla, lcnx)], colu, dt, dev, Vh=Vh)
                ev_tr[k] = ss.event(us)
                _tsqr_update(buf, lr_k, mloc, Vloc, f, [(lcnx, nloc)], colu, dt, dev, Vh=Vh)
    ss.join()


import os as _os
# stacked-R reduction of the TSQR tree by tpqrt (default) or a plain QR of the stack
_TREE_TPQRT = _os.environ.get("SLATE_AMD_TSQR_TPQRT", "1") != "0"


def _tsqr_panel(buf, mloc, pr, p, colc, pk, st, dt, dev):
    """Ranks of the panel's process column: local QR of the own panel rows,
    all-gather of the R factors, redundant QR of the stack."""
    kb, lr_k, lc_k, nmine, km = st["kb"], st["lr_k"], st["lc_k"], st["nmine"], st["km"]
    mine = buf[lr_k:mloc, lc_k:lc_k + kb]
    if nmine:
        ops.geqrf(mine, pk.get("tau")[:, 0], pk.get("T"), pk.get("V"))
    if not st["tree"]:
        return
    Rb = ops.colmajor_zeros(kb, kb, dt, dev)
    if km:
        ops.gecopy(mine[:km], Rb[:km], uplo='U')
    allR = colc.allgather(Rb.t())                     # (p, kb, kb): block r = rank r's R (transposed)
    S = ops.colmajor_empty(st["tot"], kb, dt, dev)
    for r in st["order"]:
        if st["kr"][r]:
            o = st["soff"][r]
            S[o:o + st["kr"][r]].copy_(allR[r].t()[:st["kr"][r]])
    ks = st["ks"]
    if st["kr"][st["rk"]] == kb == ks and _TREE_TPQRT:
        # the stack's top block is R_rk (upper triangular): triangle-
        # pentagonal QR (tile::tpqrt) -- the reflectors' top parts are unit
        # vectors, the triangle is never filled, and V = [I; V_B]
        Vf = ops.colmajor_zeros(st["tot"], ks, dt, dev)
        Vf[:ks].diagonal().fill_(1)
        ops.tpqrt(0, S[:ks], S[ks:], pk.get("Th"), Vf[ks:], pk.get("tauh")[:, 0])
    else:
        Vf = ops.colmajor_empty(st["tot"], ks, dt, dev)
        ops.geqrf(S, pk.get("tauh")[:, 0], pk.get("Th"), Vf)
    if km:
        o = st["soff"][pr]
        pk.get("Vh").copy_(Vf[o:o + km])
    if pr == st["rk"]:
        ops.gecopy(S[:ks], mine[:ks], uplo='U')       # R^ over R_rk; reflectors below stay


def _tsqr_update(buf, lr_k, mloc, Vl, f, ranges, comm, dt, dev, conj=True, Vh=None):
    """C = Q^H C for local columns ``ranges`` of the rows >= tile k."""
    for c0, c1 in ranges:
        if c1 > c0:
            _tsqr_apply(buf[lr_k:mloc, c0:c1], Vl, f, comm, conj, Vh=Vh)


def _tsqr_apply(C, Vl, f, comm, conj=True, Vh=None):
    """C = Q_k^H C (conj) or Q_k C with Q_k = diag(Q_r) Q^ (local block
    reflector of this rank's panel rows, then the tree on the top kr rows;
    the tree's V^H C is one all-reduce over the process column)."""
    dt, dev = C.dtype, C.device
    ct = conj_trans(dt)
    km = f["kr"]
    tr = f["tree"]
    if C.shape[1] == 0:
        return
    if conj and km and C.shape[0]:
        _apply_qh(Vl, f["T"], C, conj=True, Vh=Vh)
    if tr is not None:
        W = ops.colmajor_zeros(tr["ks"], C.shape[1], dt, dev)
        if km:
            ops.gemm(1.0, tr["V"], C[:km], 0.0, W, transA=ct)
        comm.allreduce(W)
        ops.trmm('L', 'U', ct if conj else 'N', 'N', 1.0, tr["T"], W)
        if km:
            ops.gemm(-1.0, tr["V"], W, 1.0, C[:km])
    if not conj and km and C.shape[0]:
        _apply_qh(Vl, f["T"], C, conj=False, Vh=Vh)


# ------------------------------------------------------------------ unmqr
def _same_rows(A, C):
    a, c = A.storage.bc, C.storage.bc
    return (a.mb, a.p, a.pr) == (c.mb, c.p, c.pr) and C.global_offsets()[0] == 0 and \
        a.order == c.order and A.storage.comm is C.storage.comm
def _local_V(A, k, Tk):
    """Explicit local reflectors V_r of panel k for this rank's local rows
    >= tile k (unit lower trapezoidal, kr columns: TSQR leaves one local
    block reflector per rank), available on every rank of the process row
    (bcast along the row)."""
    s = A.storage
    bc = s.bc
    nb, p, q, pr, pc = bc.nb, bc.p, bc.q, bc.pr, bc.pc
    km = Tk.get("kr", Tk["kb"])
    lr_k = min(tiles_local_before(k, p, pr) * nb, bc.mloc)
    lc_k = tiles_local_before(k, q, pc) * nb
    mloc = bc.mloc
    buf = s.local[s.origin_slot]
    nmine = max(0, mloc - lr_k)
    Vloc = ops.colmajor_empty(nmine, km, s.dtype, buf.device)
    if pc == k % q and nmine and km:
        ops.v_explicit(buf[lr_k:mloc, lc_k:lc_k + km], Vloc)
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
                _tsqr_apply(Cl, Vloc, T[k], grid.col_comm, conj=conj)
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
    """Where A's tiles live (its origin instance): new workspaces go to the
    same memory, so a host-origin matrix on a GPU machine does not get
    device-resident companions (mixed host / device operands)."""
    from ..core.storage import HOST
    st = A.storage
    d = st.device
    if st.origin_slot == HOST or d.type != "cuda":
        return -1
    return d.index if d.index is not None else 0


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
