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
  swap sequence is folded into a permutation in LDS), column-major storage,
  no RowMajor tile conversion;
* p == 1 grids (1 x q, and a single GPU) keep the whole step on device,
  stream-ordered with lookahead: panel + lookahead columns on the
  high-priority stream, trailing swaps/trsm/GEMM on the low-priority stream;
* p > 1: the panel is gathered to the diagonal owner (one col-communicator
  gather), factored there, scattered back; pivots are broadcast and the row
  exchange between process rows is one batched point-to-point step.
Pivots: `Pivots` holds 0-based GLOBAL pivot rows (LAPACK ipiv - 1).
"""
from __future__ import annotations

import torch

from .. import ops
from ..core.enums import Diag, MethodLU, Op, Option, Side, Uplo
from ..core.exceptions import SlateError
from ..core.matrix import Matrix, Pivots, TriangularMatrix
from ..core.options import get_option
from ..core.storage import DEV, l2g, local_start
from ..parallel.streams import StreamSet
from ..utils.trace import trace_block
from ._util import grid_of, target_slot, tiles_local_before


def getrf(A, pivots: Pivots, opts=None) -> int:
    """LU factorization P A = L U; returns info (0 = success)."""
    method = get_option(opts, Option.MethodLU, MethodLU.PartialPiv)
    if method == MethodLU.NoPiv:
        return getrf_nopiv(A, opts)
    if method == MethodLU.CALU:
        return getrf_tntpiv(A, pivots, opts)
    with trace_block("getrf"):
        return _getrf(A, pivots, opts, nopiv=False)


def getrf_nopiv(A, opts=None) -> int:
    with trace_block("getrf_nopiv"):
        return _getrf(A, None, opts, nopiv=True)


def getrf_tntpiv(A, pivots, opts=None) -> int:
    """CALU (tournament pivoting).  With one process row every candidate set
    is local, so the tournament reduces to partial pivoting of the local
    panel; with p > 1 the panel owner's GPU runs the final round."""
    with trace_block("getrf_tntpiv"):
        return _getrf(A, pivots, opts, nopiv=False)


def _check_view(A):
    if A.op() != Op.NoTrans or A.ioffset or A.joffset or A.row0_offset or A.col0_offset:
        raise SlateError("getrf: pass a whole (non-transposed) block-cyclic matrix")


def _getrf(A, pivots, opts, nopiv):
    s = A.storage
    if s.bc is None:
        from .aux import run_on_block_cyclic
        return run_on_block_cyclic(A, lambda B, o: _getrf(B, pivots, o, nopiv), opts)
    _check_view(A)
    bc = s.bc
    slot = target_slot(A, opts)
    buf = s.prepare_local(slot)
    if bc.mb != bc.nb:
        raise SlateError("getrf: square tiles required")
    thr = float(get_option(opts, Option.PivotThreshold, 1.0))
    la = max(0, int(get_option(opts, Option.Lookahead, 1)))
    if bc.p == 1:
        info, ipiv = _getrf_p1(A, buf, thr, la, nopiv)
    else:
        info, ipiv = _getrf_general(A, buf, thr, nopiv)
    s.mark_local_modified(slot)
    if pivots is not None and ipiv is not None:
        pivots.set(ipiv, bc.nb)
    return info


# ------------------------------------------------------------------ p == 1
def _getrf_p1(A, buf, thr, la, nopiv):
    """1 x q grid (incl. one GPU): every rank owns every row of its columns."""
    s = A.storage
    bc = s.bc
    nb, q, pc = bc.nb, bc.q, bc.pc
    m, n = s.m, s.n
    kt = min(s.mt, s.nt)
    dev = buf.device
    dt = s.dtype
    grid = grid_of(A) if q > 1 else None
    nloc = bc.nloc
    ipiv = torch.zeros(max(min(m, n), 1), dtype=torch.int64, device=dev)   # panel-relative per step
    infos = torch.zeros(max(kt, 1), dtype=torch.int64, device=dev)
    ss = StreamSet(dev, reserve_cus=64)
    ev_tr = {}
    ss.fork()
    for k in range(kt):
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
                    ops.getrf(buf[r0:m, lck:lck + kb], piv, infos[k:k + 1], threshold=thr, nopiv=nopiv)
                    Lp = buf[r0:m, lck:lck + kb]
                else:
                    Lp = ops.colmajor_empty(mk, kb, dt, dev)
                if q > 1:
                    from ..parallel.tilecomm import bcast_tile
                    if not nopiv:
                        grid.row_comm.bcast(piv, k % q)
                    bcast_tile(grid.row_comm, Lp, k % q)
            # lookahead columns; the newest one (k+la) was the first part of
            # step k-1's trailing update
            if k >= 1 and la > 0:
                ss.wait(ss.panel, ev_tr[k - 1])
            if lcla > lc1:
                _update_cols(buf, Lp, ipiv, r0, kb, m, lc1, lcla, nopiv)
            ev_panel = ss.event(ss.panel)
        us = ss.update[0]
        with ss.use(us):
            ss.wait(us, ev_panel)
            if nloc > lcla and Lp.is_cuda:
                Lp.record_stream(us)
            # column k+1+la first (next step's newest lookahead column), event,
            # then the rest
            lcnx = max(min(tiles_local_before(k + 2 + la, q, pc) * nb, nloc), lcla)
            with trace_block("getrf::trailing"):
                if lcnx > lcla:
                    _update_cols(buf, Lp, ipiv, r0, kb, m, lcla, lcnx, nopiv)
                ev_tr[k] = ss.event(us)
                if nloc > lcnx:
                    _update_cols(buf, Lp, ipiv, r0, kb, m, lcnx, nloc, nopiv)
            # swap the already-factored left columns (tiles < k).  This runs
            # on the update stream, after every trailing update that still
            # reads an earlier panel's L rows (trailing j < k overlaps panel
            # k; swapping those rows on the panel stream would race).
            if not nopiv and lck > 0:
                ops.laswp(buf[:m, 0:lck], ipiv, r0, r0 + kb, ioff=-r0)
    ss.join()
    # global pivots
    glob = ipiv.clone()
    for k in range(kt):
        r0 = k * nb
        kb = min(nb, n - r0, m - r0)
        glob[r0:r0 + kb] += r0
    if nopiv:
        glob = torch.arange(min(m, n), dtype=torch.int64, device=dev)
    info = _reduce_info(A, infos, kt, nb)
    return info, glob[:min(m, n)]


def _bcast_strided(comm, t, root):
    from ..parallel.tilecomm import bcast_tile
    return bcast_tile(comm, t, root)


def _update_cols(buf, Lp, ipiv, r0, kb, m, c0, c1, nopiv):
    """Apply step pivots, U-row trsm and the GEMM update to local columns [c0, c1)."""
    cols = buf[:m, c0:c1]
    if not nopiv:
        ops.laswp(cols, ipiv, r0, r0 + kb, ioff=-r0)
    Ukk = buf[r0:r0 + kb, c0:c1]
    ops.trsm('L', 'L', 'N', 'U', 1.0, Lp[0:kb, 0:kb], Ukk)
    if m > r0 + kb:
        ops.gemm(-1.0, Lp[kb:, :], Ukk, 1.0, buf[r0 + kb:m, c0:c1])


def _reduce_info(A, infos, kt, nb):
    iv = infos[:kt].cpu()
    info = 0
    for k in range(kt):
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
def _getrf_general(A, buf, thr, nopiv):
    """p x q grid: panel gathered to the diagonal owner's GPU, factored there,
    scattered back; distributed row exchange; SUMMA-like update."""
    s = A.storage
    bc = s.bc
    comm = s.comm
    grid = grid_of(A)
    nb, p, q, pr, pc = bc.nb, bc.p, bc.q, bc.pr, bc.pc
    m, n = s.m, s.n
    kt = min(s.mt, s.nt)
    dev = buf.device
    dt = s.dtype
    mloc, nloc = bc.mloc, bc.nloc
    glob = torch.zeros(max(min(m, n), 1), dtype=torch.int64)
    infos = torch.zeros(max(kt, 1), dtype=torch.int64, device=dev)
    for k in range(kt):
        r0 = k * nb
        kb = min(nb, n - r0, m - r0)
        rk, ck = k % p, k % q
        root = grid.rank_of(rk, ck)
        lr_k = tiles_local_before(k, p, pr) * nb          # first local row at/after tile k
        lc_k = tiles_local_before(k, q, pc) * nb
        lc1 = min(tiles_local_before(k + 1, q, pc) * nb, nloc)
        # ---- gather panel rows [r0, m) of column k to the root (col_comm)
        piv_k = torch.zeros(kb, dtype=torch.int64, device=dev)
        with trace_block("getrf::panel"):
            if pc == ck:
                myrows = buf[lr_k:mloc, lc_k:lc_k + kb]
                sizes = [max(0, _numroc(m, nb, r, p) - tiles_local_before(k, p, r) * nb) for r in range(p)]
                mx = max(sizes)
                pad = ops.colmajor_zeros(mx, kb, dt, dev)
                if myrows.shape[0]:
                    pad[:myrows.shape[0]].copy_(myrows)
                allp = grid.col_comm.allgather(pad.t().contiguous()) if p > 1 else pad.t().unsqueeze(0)
                # assemble in global order on every rank of the column (cheap, avoids a scatter step)
                P = ops.colmajor_empty(m - r0, kb, dt, dev)
                gidx, src = _panel_order(k, nb, p, m, sizes)
                for r in range(p):
                    if sizes[r]:
                        rows = allp[r][:, :sizes[r]].t()
                        P[torch.as_tensor(gidx[r], device=dev)] = rows
                if pr == rk:
                    ops.getrf(P, piv_k, infos[k:k + 1], threshold=thr, nopiv=nopiv)
                grid.col_comm.bcast(P, rk) if p > 1 else None
                grid.col_comm.bcast(piv_k, rk) if p > 1 else None
                # write my rows back (already permuted by the panel's own swaps)
                if myrows.shape[0]:
                    myrows.copy_(P[torch.as_tensor(gidx[pr], device=dev)])
                Lcol = P
            else:
                Lcol = ops.colmajor_empty(m - r0, kb, dt, dev)
        # panel + pivots along process rows
        if q > 1:
            from ..parallel.tilecomm import bcast_tile
            bcast_tile(grid.row_comm, Lcol, ck)
            grid.row_comm.bcast(piv_k, ck)
        pk = piv_k.cpu()
        glob[r0:r0 + kb] = pk + r0
        # ---- distributed row interchange on all local columns except panel col
        perm = _perm_from_pivots(pk.tolist(), r0)
        cols_mask = [(0, lc_k if pc == ck else lc1), (lc1, nloc)] if pc == ck else [(0, nloc)]
        _swap_rows_dist(buf, perm, cols_mask, nb, p, pr, mloc, grid, dt, dev)
        # ---- U row (tile row k) = L_kk^{-1} A(k, >k) on process row rk
        Ukk = ops.colmajor_empty(kb, max(nloc - lc1, 0), dt, dev)
        if pr == rk and nloc > lc1:
            lrk = tiles_local_before(k, p, pr) * nb
            ops.trsm('L', 'L', 'N', 'U', 1.0, Lcol[0:kb, 0:kb], buf[lrk:lrk + kb, lc1:nloc])
            Ukk.copy_(buf[lrk:lrk + kb, lc1:nloc])
        if p > 1 and Ukk.numel():
            grid.col_comm.bcast(Ukk, rk)
        # ---- trailing update of local rows > tile k, cols > tile k
        lr1 = tiles_local_before(k + 1, p, pr) * nb
        if mloc > lr1 and nloc > lc1:
            # Lcol rows for my local rows > tile k
            ridx = [l2g(i, nb, pr, p) - r0 for i in range(lr1, mloc)]
            Lm = ops.colmajor_empty(len(ridx), kb, dt, dev)
            ops.row_gather(Lcol, Lm, torch.as_tensor(ridx, dtype=torch.int64, device=dev))
            ops.gemm(-1.0, Lm, Ukk, 1.0, buf[lr1:mloc, lc1:nloc])
    info = _reduce_info(A, infos, kt, nb)
    return info, glob[:min(m, n)].to(dev)


def _numroc(n, nb, r, p):
    from ..core.storage import numroc
    return numroc(n, nb, r, p)


def _panel_order(k, nb, p, m, sizes):
    """Global (panel-relative) row index of each local panel row, per rank row."""
    r0 = k * nb
    gidx = {}
    for r in range(p):
        lr_k = tiles_local_before(k, p, r) * nb
        gidx[r] = [l2g(lr_k + i, nb, r, p) - r0 for i in range(sizes[r])]
    return gidx, None


def _perm_from_pivots(piv, r0):
    """Fold the swap sequence (panel-relative) into {dst_global_row: src_global_row}."""
    cur = {}
    for i, pv in enumerate(piv):
        a, b = r0 + i, r0 + pv
        if a == b:
            continue
        va, vb = cur.get(a, a), cur.get(b, b)
        cur[a], cur[b] = vb, va
    return {d: s_ for d, s_ in cur.items() if d != s_}


def _swap_rows_dist(buf, perm, col_ranges, nb, p, pr, mloc, grid, dt, dev):
    """new_row[d] = old_row[perm[d]] for the given local column ranges,
    rows distributed block-cyclically over the p process rows."""
    if not perm:
        return
    def owner(g): return (g // nb) % p
    def lrow(g): return (g // nb // p) * nb + g % nb
    for (c0, c1) in col_ranges:
        if c1 <= c0:
            continue
        cols = buf[:, c0:c1]
        w = c1 - c0
        # rows I must send: src rows I own whose destination is elsewhere
        sends, recvs, local_moves = {}, {}, []
        send_rows, recv_rows = {}, {}
        for d, s_ in sorted(perm.items()):
            od, os_ = owner(d), owner(s_)
            if od == pr and os_ == pr:
                local_moves.append((lrow(d), lrow(s_)))
            elif os_ == pr:
                send_rows.setdefault(od, []).append(lrow(s_))
            elif od == pr:
                recv_rows.setdefault(os_, []).append(lrow(d))
        for dst, rows in send_rows.items():
            t = ops.colmajor_empty(len(rows), w, dt, dev)
            ops.row_gather(cols, t, torch.as_tensor(rows, dtype=torch.int64, device=dev))
            sends[dst] = t.t().contiguous()
        for src, rows in recv_rows.items():
            recvs[src] = torch.empty((w, len(rows)), dtype=dt, device=dev)
        # local moves must read old values first
        if local_moves:
            dsts = torch.as_tensor([a for a, _ in local_moves], dtype=torch.int64, device=dev)
            srcs = torch.as_tensor([b for _, b in local_moves], dtype=torch.int64, device=dev)
            tmp = ops.colmajor_empty(len(local_moves), w, dt, dev)
            ops.row_gather(cols, tmp, srcs)
        grid.col_comm.exchange(sends, recvs)
        if local_moves:
            ops.row_scatter(tmp, cols, dsts)
        for src, rows in recv_rows.items():
            r = recvs[src].t()
            ops.row_scatter(r, cols, torch.as_tensor(rows, dtype=torch.int64, device=dev))


# ------------------------------------------------------------------ solves
def permute_rows(B, pivots: Pivots, forward=True):
    """Apply P (forward) or P^T (backward) to the rows of B (internal::permuteRows)."""
    s = B.storage
    bc = s.bc
    if bc is None:
        raise SlateError("permute_rows: block-cyclic B required")
    lb = B.local_block()
    piv = pivots.ipiv.tolist()
    npv = len(piv)
    if bc.p == 1:
        ipv = pivots.device(lb.data.device)
        if npv:
            ops.laswp(lb.data, ipv, 0, npv, ioff=0, incx=1 if forward else -1)
    else:
        grid = grid_of(B)
        # fold all swaps into one permutation (global rows)
        cur = {}
        order = range(npv) if forward else range(npv - 1, -1, -1)
        for i in order:
            a, b = i, piv[i]
            if a == b:
                continue
            va, vb = cur.get(a, a), cur.get(b, b)
            cur[a], cur[b] = vb, va
        perm = {d: s_ for d, s_ in cur.items() if d != s_}
        _swap_rows_dist(s.local[s.origin_slot], perm, [(lb.col_off, lb.col_off + lb.nloc)], bc.nb, bc.p, bc.pr,
                        bc.mloc, grid, s.dtype, lb.data.device)
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
    from .aux import allgather_dense, from_dense
    s = A.storage
    if s.comm.size == 1 or (s.bc is not None and s.bc.p * s.bc.q == 1):
        lb = A.local_block()
        n = A.n()
        F = lb.data[:n, :n]
        dev = F.device
        I = ops.colmajor_zeros(n, n, s.dtype, dev)
        ops.geset(0.0, 1.0, I)
        ipv = pivots.device(dev)
        ops.laswp(I, ipv, 0, len(pivots.ipiv), ioff=0, incx=1)
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
