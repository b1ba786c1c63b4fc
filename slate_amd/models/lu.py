"""LU family: getrf (partial pivoting), getrf_nopiv, getrf_tntpiv (CALU),
getrs, gesv, getrs_nopiv, gesv_nopiv, getri, getriOOP.

Reference: `src/getrf.cc:22-244` (panel on the HOST with MPI pivot
reductions, RowMajor device tiles for row swaps, lookahead task DAG),
`src/getrf_nopiv.cc`, `src/getrf_tntpiv.cc`, `src/getrs.cc`, `src/gesv.cc`,
`src/getri.cc`, `src/internal/internal_swap.cc:93-806`.

MI355X design:
* the panel is factored ON THE GPU (recursive LU: per-column multi-workgroup
  pivot search with last-arriver reduction + MFMA GEMM/TRSM for the blocked
  updates -- csrc/hip/getrf.hip); SLATE always factors it on the host;
* row interchanges use one permutation-gather kernel per column block (the
  swap sequence is folded into a permutation in LDS); on the GPU the 1 x q
  form factors the local block TRANSPOSED (RowMajor rows, as SLATE's GPU
  tiles, getrf.cc:51-55), so every interchange moves contiguous memory;
* p == 1 grids (1 x q, and a single GPU) keep the whole step on device,
  stream-ordered with lookahead: panel + lookahead columns on the
  high-priority stream, trailing swaps/trsm/GEMM on the low-priority stream;
* p > 1: the panel rows stay on their owners -- per column one device step
  and one all-gather of p small (|v|, row, candidate row) records over the
  column communicator, every rank picking the same pivot (_panel_pp_dist);
  pivots are broadcast and the row exchange between process rows is one
  batched point-to-point step.
Pivots: `Pivots` holds 0-based GLOBAL pivot rows (LAPACK ipiv - 1).
"""
from __future__ import annotations

import numpy as np
import torch

from .. import _native, ops
from ..core.enums import Diag, MethodLU, Op, Option, Side, Uplo
from ..core.exceptions import SlateError
from ..core.matrix import Matrix, Pivots, TriangularMatrix
from ..core.options import get_option
from ..core.storage import DEV, l2g, local_start
from ..parallel.peer import PeerMailbox
from ..parallel.streams import StreamSet
from ..utils.trace import trace_block
from ._util import grid_of, target_slot, tiles_local_before
from ..utils import watchdog as _wd


def getrf(A, pivots: Pivots, opts=None) -> int:
    """LU factorization P A = L U; returns info (0 = success).

    Memory: a host-origin matrix larger than the device budget is factored
    OUT OF CORE (left-looking block-column streaming) on ONE rank only.  On a
    p x q grid with p q > 1 every rank stages its whole local block on its
    GPU (288 GB of HBM3E per MI355X: a 2 x 4 grid holds n ~ 160k fp64 in
    core); a larger problem needs a larger grid (SLATE's workspace streaming
    for p x q, BaseMatrix.hh:2640-2781, is not implemented)."""
    method = get_option(opts, Option.MethodLU, MethodLU.PartialPiv)
    if method == MethodLU.NoPiv:
        return getrf_nopiv(A, opts)
    if method == MethodLU.CALU:
        return getrf_tntpiv(A, pivots, opts)
    with trace_block("getrf"):
        return _getrf(A, pivots, opts, mode="pp")


def getrf_nopiv(A, opts=None) -> int:
    with trace_block("getrf_nopiv"):
        return _getrf(A, None, opts, mode="nopiv")


def getrf_tntpiv(A, pivots, opts=None) -> int:
    """CALU: LU with tournament pivoting (SLATE src/getrf_tntpiv.cc,
    internal_getrf_tntpiv.cc).  Each panel's pivot rows are chosen by a
    reduction tree: every leaf (a chunk of <= ``leaf`` local rows of one
    rank) runs a partial-pivoting LU on a copy and nominates its kb pivot
    rows; a rank's nominees play off locally, then the ranks of the process
    column all-gather their nominees (p*kb rows, one collective) and every
    rank factors the stack redundantly (deterministic => identical winners
    everywhere, no broadcast of the result).  The winners are moved into the
    diagonal block by the device row exchange, L21 = A21 U11^{-1}.  Leaf size:
    Option.InnerBlocking rows (default 8 nb) or SLATE_AMD_CALU_LEAF."""
    with trace_block("getrf_tntpiv"):
        return _getrf(A, pivots, opts, mode="calu")


def _check_view(A):
    if A.op() != Op.NoTrans or A.ioffset or A.joffset or A.row0_offset or A.col0_offset:
        raise SlateError("getrf: pass a whole (non-transposed) block-cyclic matrix")


def _getrf(A, pivots, opts, mode):
    s = A.storage
    if s.bc is None:
        from .aux import run_on_block_cyclic
        return run_on_block_cyclic(A, lambda B, o: _getrf(B, pivots, o, mode), opts)
    _check_view(A)
    bc = s.bc
    slot = target_slot(A, opts)
    if bc.mb != bc.nb:
        raise SlateError("getrf: square tiles required")
    thr = float(get_option(opts, Option.PivotThreshold, 1.0))
    la = max(0, int(get_option(opts, Option.Lookahead, 1)))
    if mode == "pp":
        ooc = _maybe_ooc(A, s, slot, thr, la)
        if ooc is not None:
            if pivots is not None:
                pivots.set(ooc[1], bc.nb)
            return ooc[0]
    if getattr(s.comm, "backend", "") == "loopback" and s.comm.size > 1 and mode != "nopiv":
        # the loopback transport feeds a rank its own bytes back: broadcast
        # pivots and the peers' pivot records are then this rank's own
        # (uninitialised) buffers, and the row exchange indexes past the
        # local block (a device fault on MI355X, tools/r5/gpu_az.sh) --
        # refuse instead of faulting
        raise SlateError("pivoted getrf cannot run under the loopback transport (pivots need the peers' data)")
    buf = s.prepare_local(slot)
    if bc.p == 1 and mode != "calu":
        info, ipiv = None, None
        if _rowmajor_ok(buf, bc):
            T = _alloc_transposed(buf, bc, s.m)
            if T is not None:
                info, ipiv = _getrf_p1(A, buf, thr, la, mode == "nopiv", T=T)
        if info is None:
            info, ipiv = _getrf_p1(A, buf, thr, la, mode == "nopiv")
    else:
        import os
        leaf = int(os.environ.get("SLATE_AMD_CALU_LEAF", 0)) or \
            int(get_option(opts, Option.InnerBlocking, 0) or 0) or 8 * bc.nb
        info, ipiv = _getrf_general(A, buf, thr, la, mode, max(leaf, bc.nb))
    s.mark_local_modified(slot)
    if pivots is not None and ipiv is not None:
        pivots.set(ipiv, bc.nb)
    return info


def _maybe_ooc(A, s, slot, thr, la):
    """Host-origin matrix on one rank, larger than the device budget (or
    SLATE_AMD_OOC_COLS set): the left-looking out-of-core LU streams block
    columns instead of staging the whole local buffer (models/ooc.py).
    Returns (info, ipiv) or None for the in-core path."""
    from .ooc import getrf_ooc, ooc_applicable, ooc_block_columns
    if not ooc_applicable(A, s, slot):
        return None
    from ..core.storage import HOST
    dev = torch.device("cuda", torch.cuda.current_device())
    W = ooc_block_columns(s.m, s.n, s.bc.nb, s.dtype, dev, 5)
    if not W or W >= s.n:
        return None
    s.sync_origin()
    res = getrf_ooc(s.local[HOST][:s.m, :s.n], s.m, s.n, s.bc.nb, W, dev, thr, la)
    s.mark_local_modified(HOST)
    return res


# ------------------------------------------------------------------ p == 1
def _rowmajor_ok(buf, bc):
    """The RowMajor (transposed-storage) form of the 1 x q LU: GPU only,
    SLATE_AMD_LU_ROWMAJOR=0 turns it off."""
    import os
    return buf.is_cuda and bc.p == 1 and os.environ.get("SLATE_AMD_LU_ROWMAJOR", "1") != "0"


def _alloc_transposed(buf, bc, m):
    """nloc x m column-major workspace for the transposed local block (the
    rows of A contiguous), or None when the device cannot hold a second copy
    of the local block (then the column-major path runs)."""
    nloc = bc.nloc
    ldt = (nloc + 7) // 8 * 8
    try:
        return torch.empty((max(m, 1), ldt), dtype=buf.dtype, device=buf.device).t()[:nloc, :m]
    except torch.cuda.OutOfMemoryError:
        return None


# growth values of the explicit-inverse steps that forced a redo (tests)
LU_INV_REDO = []


def _getrf_p1(A, buf, thr, la, nopiv, T=None, no_inv=False):
    """1 x q grid (incl. one GPU): every rank owns every row of its columns.

    With ``T`` (GPU) the local block is factored TRANSPOSED, i.e. with
    RowMajor rows as SLATE does on GPUs (src/getrf.cc:51-55): T = buf^T, so
    a row interchange of A moves two contiguous columns of T (whole cache
    lines; column-major row swaps are strided 8-byte accesses, ~60 ms per
    n = 32768 factorization) and the trailing update is the NT GEMM
    T22 -= U12^T L21^T.  Each panel is copied out to a column-major block
    for the panel kernel and written back; T goes back to buf at the end."""
    s = A.storage
    bc = s.bc
    nb, q, pc = bc.nb, bc.q, bc.pc
    m, n = s.m, s.n
    kt = min(s.mt, s.nt)
    dev = buf.device
    dt = s.dtype
    grid = grid_of(A) if q > 1 else None
    nloc = bc.nloc
    rm = T is not None
    ipiv = torch.zeros(max(min(m, n), 1), dtype=torch.int64, device=dev)   # panel-relative per step
    infos = torch.zeros(max(kt, 1), dtype=torch.int64, device=dev)
    # RowMajor: buf -> T is not a separate pass in front of the
    # factorization: step 0's panel copies its columns straight from buf,
    # the panel stream transposes the lookahead columns and the update
    # stream the rest, overlapping panel 0
    upd = _update_cols_rm if rm else _update_cols
    M = T if rm else buf
    # 32 CUs: the persistent fp64 panel runs <= 32 workgroups (2 rows per thread)
    ss = StreamSet(dev, reserve_cus=32)
    ev_tr = {}
    left = []
    plans = {}
    import os
    tail = int(kt * float(os.environ.get("SLATE_AMD_LU_LEFT_TAIL", "0.6")))
    # GEMM-bound first steps (SLATE_AMD_LU_UNMASKED = fraction of the steps,
    # default 0): their trailing update runs on the unmasked diag stream --
    # all CUs -- while the panel still has slack; the CU-masked update
    # stream takes over where the panel chain becomes critical
    unmasked = int(kt * float(os.environ.get("SLATE_AMD_LU_UNMASKED", "0"))) if ss.gpu else 0
    # trailing widths of at least SLATE_AMD_LU_INV_MIN local columns solve
    # their U rows with the explicit L11 inverse (one GEMM; 0 = never;
    # dgetrf n = 32768 on one MI355X: 0 / 2048 / 8192 -> 39.4 / 40.3 / 40.4 TF/s)
    # Only the RowMajor form uses it: its input (buf) is intact until the end,
    # so a step whose inverse grew too much is redone with the trsm form.
    inv_min = int(os.environ.get("SLATE_AMD_LU_INV_MIN", "4096")) if rm and not nopiv and not no_inv else 0
    growth = torch.zeros(max(kt, 1), dtype=_native.REAL_OF[dt], device=dev)
    ss.fork()
    if rm and kt:
        # the bulk of buf -> T on the stream of step 0's trailing update,
        # concurrently with panel 0 (which reads buf itself)
        lcla0 = min(tiles_local_before(1 + la, q, pc) * nb, nloc)
        if nloc > lcla0:
            with ss.use(ss.diag if unmasked > 0 else ss.update[0]):
                ops.gecopy(buf[:m, lcla0:nloc], T[lcla0:nloc, :m], trans='T')
    for k in range(kt):
        _wd.beat(f"getrf step {k}")
        r0 = k * nb
        kb = min(nb, n - r0, m - r0)
        mk = m - r0
        own = (k % q) == pc
        lck = tiles_local_before(k, q, pc) * nb          # local col of tile k (if own)
        lc1 = tiles_local_before(k + 1, q, pc) * nb      # first local col after tile k
        lc1 = min(lc1, nloc)
        lcla = min(tiles_local_before(k + 1 + la, q, pc) * nb, nloc)
        piv = ipiv[r0:r0 + kb]
        with ss.use(ss.panel):
            # panel column k: trailing updates of steps <= k-la-1 (column k is
            # the first part of step k-la-1's trailing update)
            if k - la - 1 >= 0:
                ss.wait(ss.panel, ev_tr[k - la - 1])
            with trace_block("getrf::panel"):
                if own:
                    # the whole tile width: a wide last panel (m - r0 < tile
                    # width) also gets U12 = L11^{-1} P A12 of its extra columns
                    wk = min(nb, n - r0)
                    if rm:
                        Pk = ops.colmajor_empty(mk, wk, dt, dev)
                        if k == 0:
                            ops.gecopy(buf[r0:m, lck:lck + wk], Pk)
                        else:
                            ops.gecopy(T[lck:lck + wk, r0:m], Pk, trans='T')
                        ops.getrf(Pk, piv, infos[k:k + 1], threshold=thr, nopiv=nopiv)
                        ops.gecopy(Pk, T[lck:lck + wk, r0:m], trans='T')
                        Lp = Pk[:, 0:kb]
                    else:
                        ops.getrf(buf[r0:m, lck:lck + wk], piv, infos[k:k + 1], threshold=thr, nopiv=nopiv)
                        Lp = buf[r0:m, lck:lck + kb]
                else:
                    Lp = ops.colmajor_empty(mk, kb, dt, dev)
                if q > 1:
                    from ..parallel.tilecomm import bcast_tile
                    if not nopiv:
                        grid.row_comm.bcast(piv, k % q)
                    bcast_tile(grid.row_comm, Lp, k % q)
                # RowMajor: the step's swap sequence folded ONCE, used by every
                # column range of this step (and later by the left columns)
                sw = ipiv
                if rm and not nopiv:
                    sw = plans[k] = ops.swap_plan(ipiv, r0, r0 + kb, ioff=-r0)
            Linv = None
            if inv_min and nloc - lcla >= inv_min and kb == nb:
                Linv = _l11_inverse(Lp[0:kb, 0:kb], growth[k:k + 1])
            # lookahead columns; the newest one (k+la) was the first part of
            # step k-1's trailing update
            if k >= 1 and la > 0:
                ss.wait(ss.panel, ev_tr[k - 1])
            if rm and k == 0 and lcla > lc1:
                ops.gecopy(buf[:m, lc1:lcla], T[lc1:lcla, :m], trans='T')
            if lcla > lc1:
                upd(M, Lp, sw, r0, kb, m, lc1, lcla, nopiv, Linv)
            ev_panel = ss.event(ss.panel)
        us = ss.diag if k < unmasked else ss.update[0]
        if k == unmasked and unmasked > 0:
            ss.wait(us, ss.event(ss.diag))      # the earlier updates touch the same columns
        with ss.use(us):
            ss.wait(us, ev_panel)
            if nloc > lcla and Lp.is_cuda:
                Lp.record_stream(us)
                if Linv is not None:
                    Linv.record_stream(us)
            if rm and not nopiv:
                sw.record_stream(us)
            # column k+1+la first (next step's newest lookahead column), event,
            # then the rest
            lcnx = max(min(tiles_local_before(k + 2 + la, q, pc) * nb, nloc), lcla)
            with trace_block("getrf::trailing"):
                if lcnx > lcla:
                    upd(M, Lp, sw, r0, kb, m, lcla, lcnx, nopiv, Linv)
                ev_tr[k] = ss.event(us)
                if nloc > lcnx:
                    upd(M, Lp, sw, r0, kb, m, lcnx, nloc, nopiv, Linv)
            # swap the already-factored left columns (tiles < k).  This runs
            # on the update stream, after every trailing update that still
            # reads an earlier panel's L rows (trailing j < k overlaps panel
            # k; swapping those rows on the panel stream would race).
            # Nothing reads the left columns again before the end, so the
            # swaps are deferred into the panel-bound tail of the
            # factorization, where the update stream idles (the first ~2/3 of
            # the steps are GEMM-bound): there they are spread evenly over
            # the remaining steps, in step order.
            if not nopiv and lck > 0:
                left.append((k, r0, kb, lck))
            if k >= tail:
                todo = -(-len(left) // max(1, kt - k))
                for _ in range(min(todo, len(left))):
                    _swap_left(M, rm, m, left.pop(0), plans if rm else ipiv)
    with ss.use(ss.update[0]):
        for item in left:
            _swap_left(M, rm, m, item, plans if rm else ipiv)
    ss.join()
    if inv_min:
        from ._util import read_to_host
        lim = float(os.environ.get("SLATE_AMD_LU_INV_GROWTH", "1e6"))
        gmax = float(read_to_host(growth).max())
        if not gmax <= lim:
            LU_INV_REDO.append(gmax)
            return _getrf_p1(A, buf, thr, la, nopiv, T=T, no_inv=True)
    if rm and nloc and m:
        ops.gecopy(T, buf[:m, :nloc], trans='T')
    if nopiv:
        glob = _identity_pivots(min(m, n), dev)
    else:
        glob = _global_pivots(ipiv[:min(m, n)], nb)
    info = _reduce_info(A, infos, kt, nb)
    return info, glob


def _swap_left(M, rm, m, item, sw):
    """Step k's interchanges on the factored columns left of its panel (sw:
    the per-step plans of the RowMajor form, else the pivot vector)."""
    k, j0, jb, jc = item
    if rm:
        ops.laswp_cols_plan(M[0:jc, :m], sw[k])
    else:
        ops.laswp(M[:m, 0:jc], sw, j0, j0 + jb, ioff=-j0)


def _l11_inverse(L11, growth):
    """Explicit inverse of the unit-lower L11 for the U-row GEMM, and its
    growth max |L11^{-1}| written to the one-element device view ``growth``
    (no host sync).  |L| <= 1 under partial pivoting, but |L11^{-1}| can grow
    like 2^(kb-1), and Linv A12 then loses the backward
    stability of the substitution: the driver reads the growth vector once
    at the end and redoes the factorization with the trsm form if any step
    exceeded SLATE_AMD_LU_INV_GROWTH (default 1e6)."""
    Linv = ops.tri_inv('L', 'U', L11)
    kb = L11.shape[0]
    kmod_ = _native_mod(Linv)
    # column maxima (one workgroup per column), then the max of those
    cols = torch.empty(kb, dtype=growth.dtype, device=growth.device)
    kmod_.genorm(ops.code(Linv.dtype), 'M', 'G', 'N', 0, kb, kb, Linv.data_ptr(), ops.ld(Linv),
                 cols.data_ptr(), ops.stream(Linv))
    kmod_.genorm(ops.code(cols.dtype), 'M', 'G', 'N', 0, kb, 1, cols.data_ptr(), kb,
                 growth.data_ptr(), ops.stream(Linv))
    return Linv


def _native_mod(t):
    from .._native import kmod
    return kmod(t)


def _global_pivots(ipiv, nb):
    """Panel-relative pivots (panel k starts at row k*nb) -> global rows, as
    a pinned host tensor: read once at the end of the factorization next to
    the info values (no torch index kernels on the device; Pivots uploads it
    again, non-blocking, when a solve needs it there)."""
    from ._util import read_to_host
    h = read_to_host(ipiv).numpy()
    g = h + (np.arange(h.size, dtype=np.int64) // nb) * nb
    return torch.from_numpy(g).pin_memory() if ipiv.is_cuda else torch.from_numpy(g)


def _identity_pivots(k, dev):
    t = torch.arange(k, dtype=torch.int64)
    return t.pin_memory() if dev.type == "cuda" else t


def _update_cols(buf, Lp, ipiv, r0, kb, m, c0, c1, nopiv, Linv=None):
    """Apply step pivots, U-row trsm and the GEMM update to local columns [c0, c1).
    With Linv (the explicit inverse of the unit-lower L11, |L| <= 1 under
    partial pivoting) the U rows are one MFMA GEMM, U12 = Linv P A12, instead
    of the latency-bound blocked substitution."""
    cols = buf[:m, c0:c1]
    if not nopiv:
        ops.laswp(cols, ipiv, r0, r0 + kb, ioff=-r0)
    Ukk = buf[r0:r0 + kb, c0:c1]
    if Linv is not None:
        tmp = ops.colmajor_empty(kb, c1 - c0, Ukk.dtype, Ukk.device)
        ops.gecopy(Ukk, tmp)
        ops.gemm(1.0, Linv, tmp, 0.0, Ukk)
    else:
        ops.trsm('L', 'L', 'N', 'U', 1.0, Lp[0:kb, 0:kb], Ukk)
    if m > r0 + kb:
        ops.gemm(-1.0, Lp[kb:, :], Ukk, 1.0, buf[r0 + kb:m, c0:c1])


def _update_cols_rm(T, Lp, ipiv, r0, kb, m, c0, c1, nopiv, Linv=None):
    """_update_cols on the transposed block T = A^T: local columns [c0, c1)
    of A are rows [c0, c1) of T.  Row interchanges swap whole columns of T;
    U12^T = A12^T L11^{-T} (GEMM with the explicit inverse, else trsm from
    the right); then T22 -= U12^T L21^T, one NT GEMM."""
    cols = T[c0:c1, :m]
    if not nopiv:
        ops.laswp_cols_plan(cols, ipiv)          # ipiv: the step's folded plan
    Ut = T[c0:c1, r0:r0 + kb]
    if Linv is not None:
        tmp = ops.colmajor_empty(c1 - c0, kb, Ut.dtype, Ut.device)
        ops.gecopy(Ut, tmp)
        ops.gemm(1.0, tmp, Linv, 0.0, Ut, 'N', 'T')
    else:
        ops.trsm('R', 'L', 'T', 'U', 1.0, Lp[0:kb, 0:kb], Ut)
    if m > r0 + kb:
        ops.gemm(-1.0, Ut, Lp[kb:, :], 1.0, T[c0:c1, r0 + kb:m], 'N', 'T')


def _reduce_info(A, infos, kt, nb):
    from ._util import read_to_host
    iv = read_to_host(infos[:kt]).tolist()
    info = 0
    for k in range(kt):
        _wd.beat(f"getrf step {k}")
        if int(iv[k]) > 0:
            info = k * nb + int(iv[k])
            break
    comm = A.storage.comm
    if comm.size > 1:
        big = 1 << 62
        v = int(comm.allreduce_scalar(info if info > 0 else big, "min", torch.int64))
        info = 0 if v >= big else v
    return info


# ------------------------------------------------------------------ p > 1
_PLAN_TSRC = 1 + 1024     # int64 offset of SwapPlan.tsrc (after {nt, pad} and trow[1024])


class _Pack:
    """One flat byte buffer holding several typed column-major blocks, so a
    step's panel rows, diagonal factor and pivots travel in ONE collective
    (SLATE sends them as separate tile messages, getrf.cc:120-160)."""

    def __init__(self, parts, dev):
        off, self.spec = 0, {}
        for name, r, c, dt in parts:
            es = torch.empty(0, dtype=dt).element_size()
            off = (off + 15) // 16 * 16
            self.spec[name] = (off, r, c, dt, es)
            off += r * c * es
        self.raw = torch.empty(max(off, 16), dtype=torch.uint8, device=dev)

    def get(self, name):
        off, r, c, dt, es = self.spec[name]
        flat = self.raw[off:off + r * c * es].view(dt)
        return flat.view(c, r).t()

    def prefix(self, upto):
        """A copy of the parts before ``upto`` (one device copy), so the
        small parts can outlive the big one."""
        end = self.spec[upto][0]
        names = list(self.spec)
        out = _Pack.__new__(_Pack)
        out.spec = {k: self.spec[k] for k in names[:names.index(upto)]}
        out.raw = self.raw[:max(end, 16)].clone()
        return out


def _rows_global(lr0, lr1, nb, p, pr, r0, dev):
    """Panel-relative global rows of local rows [lr0, lr1) of process row pr
    (a device slice of a table uploaded once per geometry)."""
    from ._panels import rows_global
    return rows_global(lr0, lr1, nb, p, pr, r0, dev)


def _getrf_general(A, buf, thr, la, mode, leaf):
    """p x q grid with lookahead; the host waits only for pivots (see below).

    step k (panel column k, owned by process column ck = k % q):
      panel stream (high priority):
        [wait for column k's last update]
        panel on the ranks of column ck, one of
          pp    : all-gather the panel inside the column, every rank factors
                  it redundantly with the GPU partial-pivoting LU
                  (deterministic -> identical pivots), keeps its own rows;
          calu  : tournament pivoting (getrf_tntpiv);
          nopiv : diagonal-block LU broadcast down the column, L21 by trsm;
        ONE row broadcast of [my panel rows | L/U diagonal block | pivots]
        swap plan folded on the device from the pivots
        lookahead columns: row exchange + U-row trsm + GEMM
      update stream (low priority, own column communicator):
        rest of the trailing columns, then the left (already factored)
        columns' row exchange.
    Row exchange, two forms:
      * lookahead columns (the critical path): swap-plan driven on the
        device -- each rank packs the touched rows it owns, one all-reduce
        over the column (2kb rows x (la+1) tiles), each rank writes its new
        rows; the reduced window rows ARE the U row the update needs;
      * bulk trailing columns (off the critical path) and the left
        (factored) columns: an exact point-to-point exchange of only the
        rows that change process row (_p2p_rows), the U row then goes down
        the column in one broadcast (SLATE internal::permuteRows +
        tileBcast, getrf.cc:155-215).  Its plan needs the pivots on the
        host (RCCL point-to-point sizes are host arguments): they travel
        through a pinned buffer and are read one step late -- the host
        blocks on the PREVIOUS step's panel event (``_moves_of``) while the
        GPU still holds this step's panel, lookahead update and the previous
        bulk update in its queues, so the wait costs host run-ahead (at most
        one step), not GPU time.  A device-planned alternative exists for
        the lookahead columns (the owner-masked all-reduce above); for the
        bulk it moves 2 kb rows x every local column per step instead of
        only the rows that change process row.  The left columns'
        interchanges are applied once, after the loop, in step order."""
    s = A.storage
    bc = s.bc
    grid = grid_of(A)
    nb, p, q, pr, pc = bc.nb, bc.p, bc.q, bc.pr, bc.pc
    m, n = s.m, s.n
    kt = min(s.mt, s.nt)
    dev, dt = buf.device, s.dtype
    mloc, nloc = bc.mloc, bc.nloc
    if nb > 512:
        raise SlateError("getrf: more than one process row needs nb <= 512 (one swap plan per panel)")
    from ..core.storage import numroc
    nloc_r = [numroc(m, nb, r, p) for r in range(p)]
    ipiv = torch.zeros(max(min(m, n), 1), dtype=torch.int64, device=dev)   # panel-relative
    infos = torch.zeros(max(kt, 1), dtype=torch.int64, device=dev)
    ss = StreamSet(dev, reserve_cus=0)
    colc, rowc = grid.col_comm, grid.row_comm
    colu = grid.col_comm_u if p > 1 else colc
    ctx = dict(buf=buf, nb=nb, p=p, pr=pr, mloc=mloc, dt=dt, dev=dev, colc=colc, thr=thr, infos=infos,
               nloc_r=nloc_r, leaf=leaf, m=m)
    ev_tr = {}
    # pivots reach the host through one pinned buffer (non-blocking copy on
    # the panel stream + an event), read one step late, when the bulk of the
    # previous step's trailing update is issued -- by then the panel that
    # produced them has long finished, so the host does not stall the GPU
    pin = torch.empty(ipiv.numel(), dtype=torch.int64, pin_memory=buf.is_cuda)
    piv_ev, moves, pend = {}, {}, None
    XCHG_STATS.clear()
    # partial pivoting: the panel rows stay on their owners (per-column
    # record all-gather, _panel_pp_dist); SLATE_AMD_LU_PANEL_GATHER=1 selects
    # the all-gather + redundant factor form (_panel_pp)
    import os
    pp_dist = os.environ.get("SLATE_AMD_LU_PANEL_GATHER", "0") != "1"
    for key in LU_DIST_STATS:
        LU_DIST_STATS[key] = 0
    ss.fork()
    import os
    kstop = int(os.environ.get("SLATE_AMD_DEBUG_LU_STEPS", kt))    # debugging: stop after k steps
    us = ss.update[0]
    for k in range(min(kt, kstop)):
        _wd.beat(f"getrf step {k}")
        r0 = k * nb
        kb = min(nb, n - r0, m - r0)
        rk, ck = k % p, k % q
        lr_k = min(tiles_local_before(k, p, pr) * nb, mloc)
        # first local row after the kb-row window (a short last panel leaves
        # rows of its own tile below the window)
        lr1 = min(lr_k + kb, mloc) if pr == rk else lr_k
        lc_k = min(tiles_local_before(k, q, pc) * nb, nloc)
        lc1 = min(tiles_local_before(k + 1, q, pc) * nb, nloc)
        lcla = min(tiles_local_before(k + 1 + la, q, pc) * nb, nloc)
        lcnx = max(min(tiles_local_before(k + 2 + la, q, pc) * nb, nloc), lcla)
        nmine = mloc - lr_k
        piv = ipiv[r0:r0 + kb]
        nslot = kb if mode == "nopiv" else 2 * kb
        st = dict(k=k, r0=r0, kb=kb, rk=rk, lr_k=lr_k, lr1=lr1, lc_k=lc_k, nmine=nmine)
        with ss.use(ss.panel):
            if k - la - 1 >= 0:
                ss.wait(ss.panel, ev_tr[k - la - 1])
            pk = _Pack([("L", nmine + kb, kb, dt), ("piv", kb, 1, torch.int64)], dev)
            Lp, pv = pk.get("L"), pk.get("piv")[:, 0]
            with trace_block("getrf::panel"):
                if pc == ck:
                    {"pp": _panel_pp_dist if pp_dist else _panel_pp, "calu": _panel_calu,
                     "nopiv": _panel_nopiv}[mode](ctx, st, ipiv, Lp, pv)
                if q > 1:
                    rowc.bcast(pk.raw, ck)
                piv.copy_(pv)
                if mode != "nopiv":
                    pin[r0:r0 + kb].copy_(piv, non_blocking=True)
                    piv_ev[k] = ss.event(ss.panel)
                plan = ops.swap_plan(ipiv, r0, r0 + kb, ioff=-r0)
            Lkk = Lp[nmine:nmine + kb]
            Lbelow = Lp[lr1 - lr_k:nmine]
            upd = dict(plan=plan, nslot=nslot, kb=kb, Lkk=Lkk, Lbelow=Lbelow, rk=rk, lr_k=lr_k, lr1=lr1, k=k,
                       r0=r0, pk=pk)
            # newest lookahead column k+la: first part of step k-1's trailing update
            if k >= 1 and la > 0:
                ss.wait(ss.panel, ev_tr[k - 1])
            # (wide matrix, last panel: the tile's columns beyond kb get the
            # row exchange and the U-row solve too)
            wk = min(nb, n - r0)
            part = [(lc_k + kb, lc_k + wk)] if (pc == ck and kb < wk) else []
            _xchg_update(ctx, upd, part + [(lc1, lcla)], [], colc)
            ev_panel = ss.event(ss.panel)
        with ss.use(us):
            ss.wait(us, ev_panel)
            if buf.is_cuda:
                pk.raw.record_stream(us)
                plan.record_stream(us)
            with trace_block("getrf::trailing"):
                # the bulk of step k-1 (exact point-to-point row exchange)
                # must precede step k's first trailing column, which was part
                # of it
                if pend is not None:
                    _bulk_update(ctx, pend, mode, pin, piv_ev, moves, colu)
                _xchg_update(ctx, upd, [(lcla, lcnx)], [], colu)
                ev_tr[k] = ss.event(us)
            upd["c0"], upd["c1"] = lcnx, nloc
            pend = upd
    with ss.use(us):
        if pend is not None:
            _bulk_update(ctx, pend, mode, pin, piv_ev, moves, colu)
        # left (already factored) columns: the interchanges of every later
        # step, applied once at the end in step order (SLATE's separate
        # left-pivot task), by the same exact exchange
        if mode != "nopiv":
            for k in range(min(kt, kstop)):
                lc_k = min(tiles_local_before(k, q, pc) * nb, nloc)
                _p2p_rows(ctx, _moves_of(k, pin, piv_ev, moves, nb, min(nb, n - k * nb, m - k * nb)),
                          0, lc_k, colu, k, "left")
    ss.join()
    if mode == "nopiv":
        glob = _identity_pivots(min(m, n), dev)
    else:
        glob = _global_pivots(ipiv[:min(m, n)], nb)
    info = _reduce_info(A, infos, kt, nb)
    for peer in ctx.get("peers", ()):
        peer.check()                  # a timed-out in-kernel peer exchange fails loudly
    return info, glob


# per-step record of the point-to-point row exchanges of the last p > 1
# getrf on this rank: {"step", "part", "rows_cross", "bytes_sent", "ncols"}
XCHG_STATS = []


def _moves_of(k, pin, piv_ev, moves, nb, kb):
    """Row moves of step k as (dst, src) global rows, dst sorted: new row dst
    holds old row src.  The pivots are read from the pinned host copy once
    the panel's event has completed."""
    mv = moves.get(k)
    if mv is None:
        if piv_ev.get(k) is not None:
            piv_ev[k].synchronize()
        r0 = k * nb
        pv = pin[r0:r0 + kb].numpy()
        cur = {}
        for i in range(kb):
            a, b = r0 + i, r0 + int(pv[i])
            if a != b:
                ca, cb = cur.get(a, a), cur.get(b, b)
                cur[a], cur[b] = cb, ca
        mv = sorted((d, s_) for d, s_ in cur.items() if d != s_)
        moves[k] = mv
    return mv


def _p2p_rows(ctx, mv, c0, c1, comm, k, part):
    """Apply the row moves ``mv`` to local columns [c0, c1): rows that stay
    inside this process row move locally, rows that change process row go
    point-to-point (one batched send/recv per peer, rows in dst order on
    both sides) -- only the rows that actually change owner travel
    (internal::permuteRows, src/internal/internal_swap.cc)."""
    w = c1 - c0
    if w <= 0 or not mv:
        return
    buf, nb, p, pr, mloc, dt, dev = (ctx[x] for x in ("buf", "nb", "p", "pr", "mloc", "dt", "dev"))

    def own(g):
        return (g // nb) % p

    def loc(g):
        return (g // (nb * p)) * nb + g % nb

    sends, recvs, ld_, ls_ = {}, {}, [], []
    cross = 0
    for d, s_ in mv:
        od, os_ = own(d), own(s_)
        cross += od != os_
        if os_ == pr and od != pr:
            sends.setdefault(od, []).append(loc(s_))
        elif od == pr and os_ != pr:
            recvs.setdefault(os_, []).append(loc(d))
        elif od == pr and os_ == pr:
            ld_.append(loc(d))
            ls_.append(loc(s_))
    peers_s, peers_r = sorted(sends), sorted(recvs)
    parts = [sends[r] for r in peers_s] + [recvs[r] for r in peers_r] + [ls_, ld_]
    flat = np.concatenate([np.asarray(x, dtype=np.int64) for x in parts]) if parts else np.zeros(0, np.int64)
    nbytes = 0
    if flat.size:
        idx = torch.from_numpy(flat)
        if buf.is_cuda:
            idx = idx.pin_memory().to(dev, non_blocking=True)
        block = buf[:mloc, c0:c1]
        off, sb, rb = 0, {}, {}
        es = torch.empty(0, dtype=dt).element_size()
        for r in peers_s:
            c = len(sends[r])
            t = torch.empty(w, c, dtype=dt, device=dev)           # (w, c) = column-major c x w
            ops.row_gather(block, t.t(), idx[off:off + c])
            sb[r] = t
            off += c
            nbytes += c * w * es
        rofs = {}
        for r in peers_r:
            c = len(recvs[r])
            rb[r] = torch.empty(w, c, dtype=dt, device=dev)
            rofs[r] = (off, c)
            off += c
        nl = len(ls_)
        if nl:
            tmp = ops.colmajor_empty(nl, w, dt, dev)
            ops.row_gather(block, tmp, idx[off:off + nl])
        if sb or rb:
            comm.exchange(sb, rb)
        for r in peers_r:
            o, c = rofs[r]
            ops.row_scatter(rb[r].t(), block, idx[o:o + c])
        if nl:
            ops.row_scatter(tmp, block, idx[off + nl:off + 2 * nl])
    XCHG_STATS.append(dict(step=k, part=part, rows_cross=cross, bytes_sent=nbytes, ncols=w))


def _bulk_update(ctx, upd, mode, pin, piv_ev, moves, comm):
    """Trailing update of local columns [c0, c1) for step upd["k"]: exact row
    exchange, U row = L_kk^{-1} (window rows) on the window's process row,
    broadcast down the column, one GEMM."""
    c0, c1 = upd["c0"], upd["c1"]
    if c1 <= c0:
        return
    buf, nb, p, pr, mloc, dt, dev = (ctx[x] for x in ("buf", "nb", "p", "pr", "mloc", "dt", "dev"))
    k, kb, rk, lr_k, lr1 = upd["k"], upd["kb"], upd["rk"], upd["lr_k"], upd["lr1"]
    if mode != "nopiv":
        _p2p_rows(ctx, _moves_of(k, pin, piv_ev, moves, nb, kb), c0, c1, comm, k, "bulk")
    W = buf[lr_k:lr_k + kb, c0:c1] if pr == rk else None
    if W is not None:
        ops.trsm('L', 'L', 'N', 'U', 1.0, upd["Lkk"], W)
    U = ops.colmajor_empty(kb, c1 - c0, dt, dev)
    if W is not None:
        U.copy_(W)
    comm.bcast(U, rk)
    Lb = upd["Lbelow"]
    if Lb.shape[0]:
        ops.gemm(-1.0, Lb, U, 1.0, buf[lr1:mloc, c0:c1])


def _xchg_update(ctx, upd, ranges, swap_only, comm):
    """Row exchange of local column ranges (one all-reduce over the process
    column), then for ``ranges`` the U-row trsm and the trailing GEMM."""
    buf, nb, p, pr, mloc = ctx["buf"], ctx["nb"], ctx["p"], ctx["pr"], ctx["mloc"]
    cols = [(c0, c1) for c0, c1 in list(ranges) + list(swap_only) if c1 > c0]
    w = sum(c1 - c0 for c0, c1 in cols)
    if w == 0:
        return
    S, kb, plan = upd["nslot"], upd["kb"], upd["plan"]
    X = ops.colmajor_empty(S, w, ctx["dt"], ctx["dev"])
    off = 0
    for c0, c1 in cols:
        ops.xchg_gather(plan, buf[:mloc, c0:c1], X[:, off:off + c1 - c0], nb, p, pr)
        off += c1 - c0
    comm.allreduce(X)
    off = 0
    for c0, c1 in cols:
        ops.xchg_scatter(plan, X[:, off:off + c1 - c0], buf[:mloc, c0:c1], nb, p, pr)
        off += c1 - c0
    off = 0
    lr_k, lr1, Lbelow = upd["lr_k"], upd["lr1"], upd["Lbelow"]
    for c0, c1 in ranges:
        if c1 <= c0:
            continue
        U = X[0:kb, off:off + c1 - c0]
        ops.trsm('L', 'L', 'N', 'U', 1.0, upd["Lkk"], U)
        if pr == upd["rk"]:
            buf[lr_k:lr_k + kb, c0:c1].copy_(U)
        if Lbelow.shape[0]:
            ops.gemm(-1.0, Lbelow, U, 1.0, buf[lr1:mloc, c0:c1])
        off += c1 - c0


def _panel_pp(ctx, st, ipiv, Lp, pv):
    """Partial pivoting: the whole panel column is all-gathered inside the
    process column and factored redundantly by every rank of the column."""
    buf, nb, p, pr, mloc, dt, dev = (ctx[x] for x in ("buf", "nb", "p", "pr", "mloc", "dt", "dev"))
    r0, kb, lr_k, lc_k, nmine, k = st["r0"], st["kb"], st["lr_k"], st["lc_k"], st["nmine"], st["k"]
    m = ctx["m"]
    cnt = [max(0, ctx["nloc_r"][r] - min(tiles_local_before(k, p, r) * nb, ctx["nloc_r"][r])) for r in range(p)]
    mx = max(max(cnt), 1)
    pad = ops.colmajor_zeros(mx, kb, dt, dev)
    mine = buf[lr_k:mloc, lc_k:lc_k + kb]
    if nmine:
        pad[:nmine].copy_(mine)
    allp = ctx["colc"].allgather(pad.t())            # (p, kb, mx): block r = rank r's rows
    P = ops.colmajor_empty(m - r0, kb, dt, dev)
    for r in range(p):
        if cnt[r]:
            lr0 = tiles_local_before(k, p, r) * nb
            ops.row_scatter(allp[r].t()[:cnt[r]], P, _rows_global(lr0, lr0 + cnt[r], nb, p, r, r0, dev))
    piv = ipiv[r0:r0 + kb]
    ops.getrf(P, piv, ctx["infos"][k:k + 1], threshold=ctx["thr"])
    if nmine:
        ops.row_gather(P, mine, _rows_global(lr_k, mloc, nb, p, pr, r0, dev))
        Lp[:nmine].copy_(mine)
    Lp[nmine:nmine + kb].copy_(P[:kb])
    pv.copy_(piv)


def _panel_pp_dist(ctx, st, ipiv, Lp, pv):
    """Partial pivoting with the panel rows staying on their owners (SLATE's
    distributed panel: Tile_getrf.hh:160-447, internal_getrf.cc:20-121).

    Recursive over the panel columns.  A base block of b columns is factored
    column by column: one device step per column (apply the previous
    column's pivot + rank-1 update on my rows, then my arg-max record:
    |v|, global row, candidate row, and row j from its owner;
    csrc/hip/lu_dist.hip) and ONE all-gather of the p small records over the
    column communicator -- every rank then picks the same pivot, so no
    MAXLOC + broadcast pair is needed.  Between the halves of a recursion
    level, the left half's interchanges reach the right half's columns (and
    the right half's the left half's) by the owner-masked row exchange of
    the trailing update (xchg_gather / all-reduce / xchg_scatter: only the
    touched rows travel); U12 = L11^{-1} A12 comes out of that exchange on
    every rank, A22 -= L21 U12 is local.  No rank ever holds another rank's
    panel rows: the bytes per column are p (2b + 3) scalars, not m x nb per
    panel.  Every rank keeps the same copy T of the kb x kb top block."""
    import os
    from .._native import kmod, code, stream
    buf, nb, p, pr, mloc, dt, dev = (ctx[x] for x in ("buf", "nb", "p", "pr", "mloc", "dt", "dev"))
    r0, kb, lr_k, lc_k, nmine, k, rk = (st[x] for x in ("r0", "kb", "lr_k", "lc_k", "nmine", "k", "rk"))
    colc, thr = ctx["colc"], ctx["thr"]
    b = max(1, int(os.environ.get("SLATE_AMD_LU_DIST_B", "32")))
    W = buf[lr_k:mloc, lc_k:lc_k + kb]
    ldw = max(1, buf.stride(1))
    grow = _rows_global(lr_k, mloc, nb, p, pr, r0, dev)
    T = ops.colmajor_zeros(kb, kb, dt, dev)
    piv = ipiv[r0:r0 + kb]
    info = ctx["infos"][k:k + 1]
    part = torch.empty(2 * 1024 + 8, dtype=torch.int64, device=dev)
    mod = kmod(buf)
    cd = code(dt)

    peer = PeerMailbox.of(colc, dev) if (b <= 64 and PeerMailbox.enabled(colc, buf)) else None
    if peer is not None:
        ctx.setdefault("peers", set()).add(peer)

    def base(c0, c1):
        if peer is not None:
            # ONE persistent launch for the block: the column peers trade their
            # records through peer-mapped mailboxes (parallel/peer.py)
            G = max(1, min(64, -(-nmine // 1024)))
            mod.lu_dist_base(cd, nmine, W[:, c0:c1].data_ptr() if nmine else buf.data_ptr(), ldw, grow.data_ptr(),
                             c0, c1, T.data_ptr(), max(1, kb), piv.data_ptr(), info.data_ptr(), 0, float(thr),
                             peer.mbox.data_ptr(), p, colc.rank, peer.part.data_ptr(), peer.next_seq(c1 - c0),
                             int(pr == rk), peer.err.data_ptr(), G, stream(buf))
            LU_DIST_STATS["base_launches"] += 1
            LU_DIST_STATS["columns"] += c1 - c0
            return
        recn = 3 + 2 * (c1 - c0)
        recs = None
        for j in range(c0, c1 + 1):
            nxt = j < c1
            rec = torch.empty(recn, dtype=dt, device=dev)
            dl = j if (pr == rk and nxt) else -1
            mod.lu_dist_step(cd, nmine, W[:, c0:c1].data_ptr() if nmine else buf.data_ptr(), ldw, grow.data_ptr(),
                             c0, c1, j, recs.data_ptr() if recs is not None else 0, p, T.data_ptr(), max(1, kb),
                             piv.data_ptr(), info.data_ptr(), 0, float(thr), rec.data_ptr(), part.data_ptr(), dl,
                             stream(buf))
            if nxt:
                recs = colc.allgather(rec).contiguous()
                LU_DIST_STATS["columns"] += 1
                LU_DIST_STATS["record_allgathers"] += 1
                LU_DIST_STATS["record_bytes"] += recs.numel() * recs.element_size()

    def exchange(a, bnd, ca, cb):
        """interchanges of panel columns [a, bnd) applied to panel columns
        [ca, cb) on every rank; returns the new window rows (bnd - a)."""
        plan = ops.swap_plan(ipiv, r0 + a, r0 + bnd, ioff=-r0)
        X = ops.colmajor_empty(2 * (bnd - a), cb - ca, dt, dev)
        cols = buf[:mloc, lc_k + ca:lc_k + cb]
        ops.xchg_gather(plan, cols, X, nb, p, pr)
        colc.allreduce(X)
        ops.xchg_scatter(plan, X, cols, nb, p, pr)
        LU_DIST_STATS["exchange_bytes"] += X.numel() * X.element_size()
        LU_DIST_STATS["exchanges"] += 1
        return X[0:bnd - a]

    def rec(c0, c1):
        if c1 - c0 <= b:
            base(c0, c1)
            return
        cm = c0 + ((c1 - c0) // 2 + b - 1) // b * b
        if cm >= c1:
            cm = c1 - b
        rec(c0, cm)
        U = exchange(c0, cm, cm, c1)
        ops.trsm('L', 'L', 'N', 'U', 1.0, T[c0:cm, c0:cm], U)
        T[c0:cm, cm:c1].copy_(U)
        if pr == rk:
            W[c0:cm, cm:c1].copy_(U)
        i0 = cm if pr == rk else 0
        if nmine > i0:
            ops.gemm(-1.0, W[i0:, c0:cm], U, 1.0, W[i0:, cm:c1])
        rec(cm, c1)
        T[cm:c1, c0:cm].copy_(exchange(cm, c1, c0, cm))

    rec(0, kb)
    if nmine:
        Lp[:nmine].copy_(W)
    Lp[nmine:nmine + kb].copy_(T)
    pv.copy_(piv)


# counters of the distributed panel on this rank (tests): columns factored,
# record bytes all-gathered, exchange bytes all-reduced
LU_DIST_STATS = {"columns": 0, "record_bytes": 0, "exchange_bytes": 0, "base_launches": 0, "exchanges": 0,
                 "record_allgathers": 0}


def _panel_nopiv(ctx, st, ipiv, Lp, pv):
    """No pivoting: LU of the diagonal block on its owner, broadcast down the
    column, L21 = A21 U11^{-1} on every rank."""
    buf, p, pr, mloc, dt, dev = (ctx[x] for x in ("buf", "p", "pr", "mloc", "dt", "dev"))
    kb, lr_k, lr1, lc_k, nmine, rk, k = (st[x] for x in ("kb", "lr_k", "lr1", "lc_k", "nmine", "rk", "k"))
    D = ops.colmajor_empty(kb, kb, dt, dev)
    if pr == rk:
        Dm = buf[lr_k:lr_k + kb, lc_k:lc_k + kb]
        ops.getrf(Dm, None, ctx["infos"][k:k + 1], nopiv=True)
        D.copy_(Dm)
    if p > 1:
        ctx["colc"].bcast(D, rk)
    below = buf[lr1:mloc, lc_k:lc_k + kb]
    if below.shape[0]:
        ops.trsm('R', 'U', 'N', 'N', 1.0, D, below)
    if nmine:
        Lp[:nmine].copy_(buf[lr_k:mloc, lc_k:lc_k + kb])
    Lp[nmine:nmine + kb].copy_(D)
    pv.copy_(torch.arange(kb, dtype=torch.int64, device=dev))


def _tournament(rows, gidx, kb, thr, dev):
    """One play-off: partial-pivoting LU of a copy of ``rows`` (R x kb);
    returns the min(R, kb) winners' ORIGINAL rows, their global indices and
    the factored copy (whose top rows are the winners' L/U)."""
    R = rows.shape[0]
    c = min(R, kb)
    W = ops.colmajor_empty(R, rows.shape[1], rows.dtype, dev)
    W.copy_(rows)
    lp = torch.zeros(c, dtype=torch.int64, device=dev)
    scratch = torch.zeros(1, dtype=torch.int64, device=dev)
    ops.getrf(W, lp, scratch, threshold=thr)
    plan = ops.swap_plan(lp, 0, c, 0)
    win = plan[_PLAN_TSRC:_PLAN_TSRC + c]
    C = ops.colmajor_empty(c, rows.shape[1], rows.dtype, dev)
    ops.row_gather(rows, C, win)
    return C, gidx[win], W


def _panel_calu(ctx, st, ipiv, Lp, pv):
    buf, nb, p, pr, mloc, dt, dev, thr = (ctx[x] for x in ("buf", "nb", "p", "pr", "mloc", "dt", "dev", "thr"))
    r0, kb, lr_k, lr1, lc_k, nmine, rk, k = (st[x] for x in ("r0", "kb", "lr_k", "lr1", "lc_k", "nmine", "rk", "k"))
    leaf = ctx["leaf"]
    colc = ctx["colc"]
    mine = buf[lr_k:mloc, lc_k:lc_k + kb]
    # 1. local rounds: leaves of <= leaf rows, then the nominees play off
    if nmine:
        g_all = _rows_global(lr_k, mloc, nb, p, pr, 0, dev)
        noms, gids = [], []
        for a in range(0, nmine, leaf):
            b = min(nmine, a + leaf)
            C, g, _ = _tournament(mine[a:b], g_all[a:b], kb, thr, dev)
            noms.append(C)
            gids.append(g)
        while len(noms) > 1:
            C = ops.colmajor_empty(sum(x.shape[0] for x in noms), kb, dt, dev)
            o = 0
            for x in noms:
                C[o:o + x.shape[0]].copy_(x)
                o += x.shape[0]
            g = torch.cat(gids)
            # pairwise would need log rounds; one flat round over the
            # (few) local nominees is the same tournament with fan-in > 2
            C, g, _ = _tournament(C, g, kb, thr, dev)
            noms, gids = [C], [g]
        Cm, gm = noms[0], gids[0]
    else:
        Cm = ops.colmajor_empty(0, kb, dt, dev)
        gm = torch.zeros(0, dtype=torch.int64, device=dev)
    # 2. cross-rank round: all-gather the nominees (fixed size kb rows each)
    cnt = [min(kb, max(0, ctx["nloc_r"][r] - min(tiles_local_before(k, p, r) * nb, ctx["nloc_r"][r])))
           for r in range(p)]
    pk = _Pack([("C", kb, kb, dt), ("g", kb, 1, torch.int64)], dev)
    pC, pg = pk.get("C"), pk.get("g")[:, 0]
    if cnt[pr]:
        pC[:cnt[pr]].copy_(Cm)
        pg[:cnt[pr]].copy_(gm)
    allb = colc.allgather(pk.raw)                    # (p, nbytes)
    tot = sum(cnt)
    Stk = ops.colmajor_empty(tot, kb, dt, dev)
    Gst = torch.empty(tot, dtype=torch.int64, device=dev)
    o = 0
    for r in range(p):
        if cnt[r]:
            rb = _Pack.__new__(_Pack)
            rb.spec, rb.raw = pk.spec, allb[r]
            Stk[o:o + cnt[r]].copy_(rb.get("C")[:cnt[r]])
            Gst[o:o + cnt[r]].copy_(rb.get("g")[:cnt[r], 0])
            o += cnt[r]
    # 3. final round, redundantly on every rank of the column
    sp = torch.zeros(kb, dtype=torch.int64, device=dev)
    ops.getrf(Stk, sp, ctx["infos"][k:k + 1], threshold=thr)
    splan = ops.swap_plan(sp, 0, kb, 0)
    sel = Gst[splan[_PLAN_TSRC:_PLAN_TSRC + kb]]
    piv = ipiv[r0:r0 + kb]
    ops.sel_to_ipiv(sel, r0, piv)
    # 4. winners into the diagonal block (device row exchange on the panel column)
    plan = ops.swap_plan(ipiv, r0, r0 + kb, ioff=-r0)
    X = ops.colmajor_empty(2 * kb, kb, dt, dev)
    ops.xchg_gather(plan, buf[:mloc, lc_k:lc_k + kb], X, nb, p, pr)
    colc.allreduce(X)
    ops.xchg_scatter(plan, X, buf[:mloc, lc_k:lc_k + kb], nb, p, pr)
    LU = Stk[:kb]
    if pr == rk:
        buf[lr_k:lr_k + kb, lc_k:lc_k + kb].copy_(LU)
    below = buf[lr1:mloc, lc_k:lc_k + kb]
    if below.shape[0]:
        ops.trsm('R', 'U', 'N', 'N', 1.0, LU, below)
    if nmine:
        Lp[:nmine].copy_(mine)
    Lp[nmine:nmine + kb].copy_(LU)
    pv.copy_(piv)


def permute_rows(B, pivots: Pivots, forward=True):
    """Apply P (forward) or P^T (backward) to the rows of B (internal::permuteRows).
    p > 1: the swap sequence is folded on the device in chunks of <= 512
    swaps and applied by the same owner-masked exchange as getrf (one column
    all-reduce per chunk, no host round trip)."""
    s = B.storage
    bc = s.bc
    if bc is None:
        raise SlateError("permute_rows: block-cyclic B required")
    lb = B.local_block()
    npv = pivots.size
    if bc.p == 1:
        ipv = pivots.device(lb.data.device)
        if npv:
            ops.laswp(lb.data, ipv, 0, npv, ioff=0, incx=1 if forward else -1)
    elif npv:
        grid = grid_of(B)
        buf = s.local[s.origin_slot]
        ipv = pivots.device(buf.device)
        cols = buf[:bc.mloc, lb.col_off:lb.col_off + lb.nloc]
        chunks = [(a, min(npv, a + 512)) for a in range(0, npv, 512)]
        for a, b in (chunks if forward else chunks[::-1]):
            plan = ops.swap_plan(ipv, a, b, 0, incx=1 if forward else -1)
            if cols.shape[1]:
                X = ops.colmajor_empty(2 * (b - a), cols.shape[1], s.dtype, buf.device)
                ops.xchg_gather(plan, cols, X, bc.nb, bc.p, bc.pr)
            else:
                X = ops.colmajor_empty(2 * (b - a), 0, s.dtype, buf.device)
            grid.col_comm.allreduce(X) if X.numel() else None
            if cols.shape[1]:
                ops.xchg_scatter(plan, X, cols, bc.nb, bc.p, bc.pr)
    s.mark_local_modified(s.origin_slot)
    return B


def getrs(A, pivots, B, opts=None):
    """Solve op(A) X = B with the LU factors of A."""
    from .blas3 import trsm
    L = TriangularMatrix(Uplo.Lower, A, diag=Diag.Unit)
    U = TriangularMatrix(Uplo.Upper, A, diag=Diag.NonUnit)
    if A.op() == Op.NoTrans:
        permute_rows(B, pivots, forward=True)
        trsm(Side.Left, 1.0, L, B, opts)
        trsm(Side.Left, 1.0, U, B, opts)
    else:
        # A^T X = B:  U^T L^T P X = B
        Lt = L.transpose() if A.op() == Op.Trans else L.conj_transpose()
        Ut = U.transpose() if A.op() == Op.Trans else U.conj_transpose()
        Lt._uplo, Ut._uplo = Uplo.Lower, Uplo.Upper
        Lt._uplo = Uplo.Lower
        trsm(Side.Left, 1.0, _tri_of(A, Uplo.Upper, Diag.NonUnit, A.op()), B, opts)
        trsm(Side.Left, 1.0, _tri_of(A, Uplo.Lower, Diag.Unit, A.op()), B, opts)
        permute_rows(B, pivots, forward=False)
    return 0


def _tri_of(A, uplo, diag, op):
    base = A if A.op() == Op.NoTrans else (A.transpose() if A.op() == Op.Trans else A.conj_transpose())
    T = TriangularMatrix(uplo, base, diag=diag)
    return T.transpose() if op == Op.Trans else T.conj_transpose()


def gesv(A, pivots, B, opts=None) -> int:
    method = get_option(opts, Option.MethodLU, MethodLU.PartialPiv)
    if method == MethodLU.RBT:
        from .mixed import gesv_rbt
        return gesv_rbt(A, B, opts)
    if method == MethodLU.NoPiv:
        return gesv_nopiv(A, B, opts)
    info = getrf(A, pivots, opts)
    if info == 0:
        getrs(A, pivots, B, opts)
    return info


def getrs_nopiv(A, B, opts=None):
    from .blas3 import trsm
    if A.op() == Op.NoTrans:
        trsm(Side.Left, 1.0, TriangularMatrix(Uplo.Lower, A, diag=Diag.Unit), B, opts)
        trsm(Side.Left, 1.0, TriangularMatrix(Uplo.Upper, A, diag=Diag.NonUnit), B, opts)
    else:
        trsm(Side.Left, 1.0, _tri_of(A, Uplo.Upper, Diag.NonUnit, A.op()), B, opts)
        trsm(Side.Left, 1.0, _tri_of(A, Uplo.Lower, Diag.Unit, A.op()), B, opts)
    return 0


def gesv_nopiv(A, B, opts=None) -> int:
    info = getrf_nopiv(A, opts)
    if info == 0:
        getrs_nopiv(A, B, opts)
    return info


def getri(A, pivots, opts=None) -> int:
    """In-place inverse from the LU factors: inv(A) = inv(U) inv(L) P."""
    s = A.storage
    if s.comm.size == 1 or (s.bc is not None and s.bc.p * s.bc.q == 1):
        lb = A.local_block()
        n = A.n()
        F = lb.data[:n, :n]
        dev = F.device
        I = ops.colmajor_zeros(n, n, s.dtype, dev)
        ops.geset(0.0, 1.0, I)
        ipv = pivots.device(dev)
        ops.laswp(I, ipv, 0, pivots.size, ioff=0, incx=1)
        ops.trsm('L', 'L', 'N', 'U', 1.0, F, I)
        ops.trsm('L', 'U', 'N', 'N', 1.0, F, I)
        F.copy_(I)
        s.mark_local_modified(s.origin_slot)
        return 0
    # distributed: solve A X = I with the factors
    Id = A.emptyLike()
    Id.insertLocalTiles(device=s.device if s.device.type == "cuda" else -1)
    from .aux import set as aset
    aset(0.0, 1.0, Id)
    getrs(A, pivots, Id, opts)
    from .aux import copy
    copy(Id, A)
    return 0


def getriOOP(A, pivots, B, opts=None) -> int:
    """Out-of-place inverse: B = inv(A)."""
    from .aux import copy, set as aset
    aset(0.0, 1.0, B)
    getrs(A, pivots, B, opts)
    return 0
