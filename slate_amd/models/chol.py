"""Cholesky family: potrf, potrs, posv, potri (+ mixed precision in mixed.py).

Reference: `src/potrf.cc:22-210` (right-looking tiled Cholesky with
lookahead over an OpenMP task DAG), `src/potrs.cc`, `src/posv.cc:70-95`,
`src/potri.cc`.

MI355X design of the distributed potrf (Lower, p x q block-cyclic):

  step k (tile column g):
    panel stream (high priority):
      [wait trailing update of step k-la]   column g is now final
      potrf(A_gg)                 one workgroup, tile in L2        (diag owner)
      bcast A_gg down the column  col_comm (RCCL)                  (p > 1)
      trsm  A_{>g,g} A_gg^{-H}    blocked: small-LDS solve + MFMA GEMMs
      bcast panel along the row   row_comm (RCCL)                  (q > 1)
      p bcasts down the column of exactly the panel tiles column pc needs,
      one row-gather kernel assembles them in global order          (p > 1)
      lookahead: update tile columns g+1..g+la (ONE masked GEMM)
    update stream (low priority):
      trailing update of all remaining local columns: ONE MFMA GEMM over
      the rank's contiguous local buffer with the lower-triangle mask
      evaluated in global coordinates (SLATE: per-tile batched herk/gemm
      device regions, src/internal/internal_herk.cc:350-535).

No host synchronisation inside the factorization: per-step info values
are written by the tile kernel to a device vector and reduced once at the
end (SLATE: device_info copy + queue sync per panel, internal_potrf.cc:76).
"""
from __future__ import annotations

import os

import torch

from .. import ops
from ..core.enums import Diag, Op, Option, Side, Target, Uplo
from ..core.exceptions import SlateError
from ..core.matrix import HermitianMatrix, Matrix, TriangularMatrix
from ..core.options import get_option
from ..core.storage import DEV, HOST
from ..parallel.streams import StreamSet
from ..utils.trace import trace_block
from ._panels import assemble_cols, plan_col_gathers_steps
from ._util import conj_trans, grid_of, target_slot, tiles_local_before
from ..utils import watchdog as _wd


def _upper_to_lower(A, fn, opts):
    """Run a Lower-only algorithm on an Upper-stored Hermitian matrix via its
    conjugate transpose (SLATE potrf.cc:45-47 does the same view trick)."""
    from .aux import copy_conj_transpose
    L = HermitianMatrix(Uplo.Lower, A.emptyLike())
    L.insertLocalTiles(device=A.storage.device if target_slot(A, opts) == DEV else -1)
    copy_conj_transpose(A, L)
    info = fn(L, opts)
    copy_conj_transpose(L, A)
    return info


def potrf(A, opts=None) -> int:
    """Cholesky factorization A = L L^H (or U^H U). Returns info (0 = ok).

    Memory: a host-origin matrix larger than the device budget is factored
    OUT OF CORE (left-looking block-column streaming) on ONE rank only.  On a
    p x q grid with p q > 1 every rank stages its whole local block on its
    GPU (288 GB of HBM3E per MI355X: a 2 x 4 grid holds n ~ 160k fp64 in
    core); a larger problem needs a larger grid (SLATE's workspace streaming
    for p x q, BaseMatrix.hh:2640-2781, is not implemented)."""
    if A.uplo() == Uplo.Upper and A.op() == Op.NoTrans:
        return _upper_to_lower(A, potrf, opts)
    if A.op() != Op.NoTrans:
        # A^H of an Upper matrix is Lower: factor the stored Upper directly
        raise SlateError("potrf: pass the matrix itself, not a transposed view")
    with trace_block("potrf"):
        return _potrf_lower(A, opts)


def _maybe_ooc(A, s, slot, la):
    """Host-origin matrix, device target, one rank, larger than the device
    budget (or SLATE_AMD_OOC_COLS set): the out-of-core left-looking
    factorization streams block columns instead of staging the whole local
    buffer (models/chol_ooc.py).  Returns info, or None for the in-core path."""
    from ..core.storage import DEV, HOST
    bc = s.bc
    if slot != DEV or s.origin_slot != HOST or bc.p * bc.q != 1 or A.ioffset or A.joffset \
            or A.row0_offset or A.col0_offset or A.last_mb is not None or A.n() != s.n:
        return None
    from .chol_ooc import ooc_columns, potrf_ooc
    dev = torch.device("cuda", torch.cuda.current_device())
    n = s.n
    W = ooc_columns(n, bc.nb, s.dtype, dev)
    if not W or W >= n:
        return None
    s.sync_origin()
    info = potrf_ooc(s.local[HOST][:n, :n], n, bc.nb, W, dev, la)
    s.mark_local_modified(HOST)
    return info


def _potrf_lower(A, opts):
    s = A.storage
    bc = s.bc
    if bc is None:
        from .aux import run_on_block_cyclic
        return run_on_block_cyclic(A, _potrf_lower, opts)
    slot = target_slot(A, opts)
    la = max(0, int(get_option(opts, Option.Lookahead, 1)))
    ooc = _maybe_ooc(A, s, slot, la)
    if ooc is not None:
        return ooc
    buf = s.prepare_local(slot)
    dev = buf.device
    nb, p, q, pr, pc = bc.nb, bc.p, bc.q, bc.pr, bc.pc
    dtype = s.dtype
    ct = conj_trans(dtype)
    grid = grid_of(A) if s.comm.size > 1 else None
    g0 = A.ioffset
    if A.row0_offset or A.col0_offset or A.ioffset != A.joffset:
        raise SlateError("potrf: view must start on a diagonal tile boundary")
    nt = A.mt()
    gend = g0 + nt                                  # one past last storage tile
    R_end = s.row_offsets[gend] if A.last_mb is None else s.row_offsets[gend - 1] + A.last_mb
    lr_end = _lstart(R_end, nb, pr, p)
    lc_end = _lstart(R_end, nb, pc, q)
    ss = StreamSet(dev, reserve_cus=0)   # one-CU panel kernels: no reserved CUs (measured: 49.0 vs 45.1 TF/s with 32)
    infos = torch.zeros(max(nt, 1), dtype=torch.int64, device=dev)
    group = int(os.environ.get("SLATE_AMD_POTRF_GROUP", "2"))
    if p == 1 and q == 1 and group > 1 and nt > 2:
        if get_option(opts, Option.UseGraph, False) and buf.is_cuda:
            infos = _potrf_graph_run(A, s, buf, nb, g0, nt, R_end, la, group, ss, ct, dev)
        else:
            _potrf_1x1_grouped(A, s, buf, nb, g0, nt, R_end, la, group, ss, infos, ct, dev)
        s.mark_local_modified(slot)
        return _potrf_info(s, infos, g0, nt)
    # per step: the lookahead tiles' transposed rows (critical path) and the
    # rest (the trailing update's operand); both gathered from the panel
    # stream.  Plans are cached per geometry (_panels.plan_col_gathers_steps).
    plans = plan_col_gathers_steps(s.tileMb, g0, nt, nb, p, q, pc, dev, split=la) if (p > 1 or q > 1) else None
    # diag-first (needs a lookahead column): right after the panel solve of
    # step t, the rows of tile g+1 travel to the next diagonal owner, which
    # updates and factors A(g+1, g+1) on the diag stream while the big
    # panel broadcast and the lookahead update proceed on the panel stream
    diag_first = la >= 1 and nt > 1 and os.environ.get("SLATE_AMD_POTRF_DIAGFIRST", "1") != "0"
    ev_diag = {}
    ev_tr = {}
    # tile rows per row-broadcast chunk after the first (SLATE_AMD_POTRF_CHUNK):
    # 16 -- under the in-DAG link model (loopback_critpath.py --link, 2x4 at
    # n = 32768) 4-tile chunks cost 49.6 / 88.7 ms (10 us, 150 GB/s / 25 us,
    # 50 GB/s), 8: 47.5 / 84.5, 16: 45.9 / 82.6, 32-64: the same as 16
    chunk_tiles = max(1, int(os.environ.get("SLATE_AMD_POTRF_CHUNK", "16")))
    esz = torch.empty(0, dtype=dtype).element_size()
    # step pairs (SLATE_AMD_POTRF_PAIR=1, lookahead 1 with diag-first): the
    # trailing update of the pair's first step is deferred and applied with
    # the second's as ONE K = 2 nb GEMM; the second step's lookahead column
    # and diagonal tile take the deferred panel as an extra K = nb product
    # (panel / diag streams, off the big GEMM).  Opt-in: once the exact
    # staircase grid stopped losing L2 reuse on tall / wide local blocks
    # (K = 512 trailing GEMM of 1x2 rank 0 at n = 32768: 42 -> 59 TF/s), the
    # extra panel-stream products cost more than K = 1024 gains -- loopback
    # n = 32768 rank 0: 1x2 118.8 ms off vs 124.0 on, 2x2 64.4 vs 68.2, 2x4
    # 38.8 vs 41.4, 2x1 114.8 vs 112.3 (profiles/r5/critpath_2x4.md)
    pair = la == 1 and diag_first and os.environ.get("SLATE_AMD_POTRF_PAIR", "0") == "1"
    pend = None
    POTRF_BCAST_STATS.clear()
    ss.fork()
    for t in range(nt):
        _wd.beat(f"potrf step {t}")
        st_step = {"step": t, "row_bytes_first": 0, "col_bytes_first": 0, "row_msgs": 0, "row_bytes": 0}
        POTRF_BCAST_STATS.append(st_step)
        g = g0 + t
        kb = s.tileMb(g) if t < nt - 1 or A.last_mb is None else A.last_mb
        lrg = tiles_local_before(g, p, pr) * nb
        lcg = tiles_local_before(g, q, pc) * nb
        lr1 = tiles_local_before(g + 1, p, pr) * nb
        lc1 = tiles_local_before(g + 1, q, pc) * nb
        lr1, lc1 = min(lr1, lr_end), min(lc1, lc_end)
        own_col = (g % q) == pc
        own_diag = own_col and (g % p) == pr
        prev, pend = pend, None
        defer = pair and prev is None and t + 1 < nt
        with ss.use(ss.panel):
            # panel column g: every trailing update of steps <= t-la-1 (the
            # first column of step t-la-1's trailing update is this one)
            if t - la - 1 >= 0:
                ss.wait(ss.panel, ev_tr[t - la - 1])
            with trace_block("potrf::panel"):
                if own_diag:
                    if t in ev_diag:
                        ss.wait(ss.panel, ev_diag.pop(t))       # factored during step t-1 (diag-first)
                    else:
                        ops.potrf('L', buf[lrg:lrg + kb, lcg:lcg + kb], infos[t:t + 1])
                # diagonal tile -> column
                if own_col:
                    if p > 1:
                        D = ops.colmajor_empty(kb, kb, dtype, dev)
                        if own_diag:
                            D.copy_(buf[lrg:lrg + kb, lcg:lcg + kb])
                        grid.col_comm.bcast(D, g % p)
                    else:
                        D = buf[lrg:lrg + kb, lcg:lcg + kb]
                    P = buf[lr1:lr_end, lcg:lcg + kb]
                    if P.shape[0]:
                        ops.trsm('R', 'L', ct, 'N', 1.0, D, P)
                # panel -> row, TILE-GRANULAR (SLATE's per-tile listBcastMT,
                # potrf.cc:122-132): chunk 0 = the first tile row(s) of this
                # process row -- the lookahead tiles' rows on their owners and
                # the next diagonal tile's rows -- then chunks of CH tile rows,
                # all on the diag stream (the row communicator's stream) while
                # the panel stream runs the lookahead GEMM row block of each
                # chunk as it lands: the GEMM starts after ~one tile instead of
                # the whole nrow x kb panel (67 MB per early step at n = 32768
                # on 2 x 4).
                nrow = lr_end - lr1
                chunks = _row_chunks(nrow, nb, la, p, chunk_tiles)
                Prow, land, first = _bcast_panel_rows(grid, q, buf, lr1, lr_end, lcg, kb, own_col, g % q, chunks,
                                                      dtype, dev, st_step, ss)
                if chunks:
                    land(0)
                # diag-first: the next diagonal tile, on its own stream; its
                # rows are the first rows of chunk 0 on the owning process row
                kb1 = 0
                if diag_first and t + 1 < nt:
                    g1 = g + 1
                    kb1 = s.tileMb(g1) if t + 1 < nt - 1 or A.last_mb is None else A.last_mb
                    if pr == g1 % p:
                        # chunk 0 itself, on the diag stream right behind its
                        # broadcast (q == 1: the panel rows)
                        Pt = first[0:kb1]
                        ev_solve = ss.event(ss.panel)
                        with ss.use(ss.diag):
                            ss.wait(ss.diag, ev_solve)
                            # A(g+1, g+1) must also hold every earlier trailing
                            # update: with la < 2 column g+1 was not a lookahead
                            # column of step t-1, so its update by panel t-1
                            # ran on the update stream (first part, ev_tr[t-1])
                            if la < 2 and t >= 1:
                                ss.wait(ss.diag, ev_tr[t - 1])
                            if Pt.is_cuda and q > 1:
                                first.record_stream(ss.diag)
                            with trace_block("potrf::diag_first"):
                                if pc == g1 % q:
                                    D1 = buf[lr1:lr1 + kb1, lc1:lc1 + kb1]
                                    if prev is not None:
                                        Pp = prev["Prow"][lr1 - prev["lr1"]:lr1 - prev["lr1"] + kb1]
                                        ops.gemm(-1.0, Pp, Pp, 1.0, D1, 'N', ct, (1, 1 << 40, 1, 0, 1, 0, 0, 0, 0))
                                    ops.gemm(-1.0, Pt, Pt, 1.0, D1, 'N', ct, (1, 1 << 40, 1, 0, 1, 0, 0, 0, 0))
                                    ops.potrf('L', D1, infos[t + 1:t + 2])
                                    ev_diag[t + 1] = ss.event(ss.diag)
                # panel -> column: the lookahead tiles' rows now (they are in
                # chunk 0), the rest after the lookahead update
                if plans is not None:
                    Lla = assemble_cols(plans[t][0], Prow, grid, p, kb, dtype, dev)
                    st_step["col_bytes_first"] = sum(plans[t][0][0][r][1] for r in range(p)) * kb * esz
                else:
                    Lla = Lcol = Prow
            # lookahead columns g+1 .. g+la
            lc_la = min(tiles_local_before(g + 1 + la, q, pc) * nb, lc_end)
            # the newest lookahead column g+la was in step t-1's trailing
            # update (its first part): wait for exactly that part
            if t >= 1 and la > 0:
                ss.wait(ss.panel, ev_tr[t - 1])
            diag_done = bool(kb1 and t + 1 in ev_diag and pr == (g + 1) % p and pc == (g + 1) % q)
            # the lookahead column's products: the deferred panel of the
            # pair's first step (its rows from local row lr1, its transposed
            # rows from local column lc1), then this step's panel
            srcs = [(Prow, Lla, 0, 0)]
            if prev is not None:
                srcs.insert(0, (prev["Prow"], prev["Lcol"], lr1 - prev["lr1"], lc1 - prev["loff"]))
            for ci, (ra, rb) in enumerate(chunks):
                if ci:
                    land(ci)
                if lc_la <= lc1:
                    continue
                for Pk, Lk, o, lo in srcs:
                    if diag_done:
                        # the diagonal tile of g+1 is already updated and factored:
                        # its column below it, then the other lookahead columns
                        a1 = max(ra, kb1)
                        if rb > a1:
                            ops.gemm(-1.0, Pk[o + a1:o + rb], Lk[lo:lo + kb1], 1.0, buf[lr1 + a1:lr1 + rb, lc1:lc1 + kb1],
                                     'N', ct, (1, nb, p, pr, q, pc, lr1 + a1, lc1, 0))
                        if lc_la > lc1 + kb1:
                            ops.gemm(-1.0, Pk[o + ra:o + rb], Lk[lo + kb1:lo + lc_la - lc1], 1.0,
                                     buf[lr1 + ra:lr1 + rb, lc1 + kb1:lc_la], 'N', ct,
                                     (1, nb, p, pr, q, pc, lr1 + ra, lc1 + kb1, 0))
                    else:
                        mask = (1, nb, p, pr, q, pc, lr1 + ra, lc1, 0)
                        ops.gemm(-1.0, Pk[o + ra:o + rb], Lk[lo:lo + lc_la - lc1], 1.0, buf[lr1 + ra:lr1 + rb, lc1:lc_la],
                                 'N', ct, mask)
            ev_panel = ss.event(ss.panel)
        us = ss.update[0]
        # the trailing update's transposed rows: gathered from the UPDATE
        # stream over the grid's second column communicator (col_comm_u, one
        # issue order on every rank), so the next step's panel no longer
        # queues behind the step's biggest column broadcast (2x4 at n =
        # 32768 under the in-DAG link model: profiles/r5/critpath_2x4.md);
        # -- when q > 1 (one process column: the update stream already carries
        # all the GEMM work, and 2x1 lost 123 -> 142 ms with it);
        # SLATE_AMD_POTRF_LCOL_U=0|1 forces the panel stream / update stream
        if plans is not None:
            lcol_u = os.environ.get("SLATE_AMD_POTRF_LCOL_U", "1" if q > 1 else "0") != "0"
            st_l = us if lcol_u else ss.panel
            with ss.use(st_l):
                if lcol_u:
                    ss.wait(us, ev_panel)
                    if Prow.is_cuda:
                        Prow.record_stream(us)
                Lcol = assemble_cols(plans[t][1], Prow, grid, p, kb, dtype, dev,
                                     comm=grid.col_comm_u if lcol_u else None)
                if not lcol_u:
                    ev_panel = ss.event(ss.panel)
            loff = lc_la            # Lcol row 0 = local column lc_la
        else:
            loff = lc1
        if defer:
            # the pair's first step: its trailing update waits for the second
            pend = {"Prow": Prow, "Lcol": Lcol, "lr1": lr1, "loff": loff, "lcg": lcg, "own_col": own_col}
            if Prow.is_cuda:
                for x in (Prow, Lcol):
                    x.record_stream(ss.diag)
                    x.record_stream(us)
            with ss.use(us):
                ev_tr[t] = ss.event(us)
            continue
        if prev is not None and nrow and lc_end > lc_la:
            # K = 2 kb operands: [deferred panel | this panel], rows from lr1,
            # transposed rows from local column lc_la (= loff)
            with ss.use(us):
                ss.wait(us, ev_panel)
                Pp, Lp = prev["Prow"], prev["Lcol"]
                if q == 1:
                    # both panel columns are local and adjacent
                    Prow = buf[lr1:lr_end, prev["lcg"]:lcg + kb]
                else:
                    Pc = ops.colmajor_empty(nrow, Pp.shape[1] + kb, dtype, dev)
                    Pc[:, :Pp.shape[1]].copy_(Pp[lr1 - prev["lr1"]:])
                    Pc[:, Pp.shape[1]:].copy_(Prow)
                    Prow = Pc
                Lc = ops.colmajor_empty(lc_end - loff, Lp.shape[1] + kb, dtype, dev)
                Lc[:, :Lp.shape[1]].copy_(Lp[loff - prev["loff"]:])
                Lc[:, Lp.shape[1]:].copy_(Lcol[:lc_end - loff])
                Lcol = Lc
        # trailing update
        with ss.use(us):
            ss.wait(us, ev_panel)
            # split: column g+1+la first (the next step's newest lookahead
            # column and, la steps later, a panel), event, then the rest
            lc_nx = min(tiles_local_before(g + 2 + la, q, pc) * nb, lc_end)
            lc_nx = max(lc_nx, lc_la)
            if Prow.is_cuda and lc_end > lc_la and nrow:
                Prow.record_stream(us)
                if Lcol is not Prow:
                    Lcol.record_stream(us)
            with trace_block("potrf::trailing"):
                for c0, c1 in ((lc_la, lc_nx), (lc_nx, lc_end)):
                    if c1 > c0 and nrow:
                        mask = (1, nb, p, pr, q, pc, lr1, c0, 0)
                        ops.gemm(-1.0, Prow, Lcol[c0 - loff:c1 - loff], 1.0, buf[lr1:lr_end, c0:c1],
                                 'N', ct, mask)
                    if c0 == lc_la:
                        ev_tr[t] = ss.event(us)
    ss.join()
    s.mark_local_modified(slot)
    return _potrf_info(s, infos, g0, nt)


# per step of the last distributed potrf on this rank: bytes of the row
# broadcast the first lookahead GEMM waits for (chunk 0), of the column
# broadcasts assembling its operand, and the whole row broadcast
POTRF_BCAST_STATS = []


def _row_chunks(nrow, nb, la, p, ch):
    """Row ranges of the tile-granular panel broadcast: chunk 0 = the tiles
    holding this process row's lookahead rows (ceil(la / p) tile rows, at
    least one), then ``ch`` tile rows per chunk."""
    if nrow <= 0:
        return []
    first = min(nrow, nb * max(1, -(-la // p)))
    out, a = [(0, first)], first
    while a < nrow:
        b = min(nrow, a + ch * nb)
        out.append((a, b))
        a = b
    return out


# SLATE_AMD_BCAST_SA=1: the row broadcasts of the panel (q >= 3) as a direct
# scatter + all-gather (Comm.bcast_sa): 2 B / q per xGMI link instead of B
# (per-link projection: profiles/r6/critpath_2x4_links.md)
_BCAST_SA = __import__("os").environ.get("SLATE_AMD_BCAST_SA", "0") == "1"


def _bcast_panel_rows(grid, q, buf, lr1, lr_end, lcg, kb, own_col, root, chunks, dtype, dev, st, ss):
    """Issue every chunk's row broadcast on the DIAG stream -- the row
    communicator's one stream (torch runs a synchronous RCCL collective on
    the issuing stream, profiles/r4/nccl_stream_probe.txt, so a
    communicator used from one stream adds no hardware queue and its
    collectives keep one order on every rank); the owner sends contiguous
    copies of its rows.  Returns (Prow, land, first): land(i) makes the
    panel stream wait for chunk i and places it in Prow; ``first`` is chunk
    0's buffer, on the diag stream.  q == 1: Prow is the buffer itself."""
    if q == 1:
        P = buf[lr1:lr_end, lcg:lcg + kb]
        return P, (lambda i: None), P
    nrow = lr_end - lr1
    Prow = buf[lr1:lr_end, lcg:lcg + kb] if own_col else ops.colmajor_empty(nrow, kb, dtype, dev)
    esz = torch.empty(0, dtype=dtype).element_size()
    pend = []
    for ci, (a, b) in enumerate(chunks):
        cb = ops.colmajor_empty(b - a, kb, dtype, dev)
        if own_col:
            cb.copy_(buf[lr1 + a:lr1 + b, lcg:lcg + kb])
        ev_src = ss.event(ss.panel)
        with ss.use(ss.diag):
            ss.wait(ss.diag, ev_src)
            if cb.is_cuda:
                cb.record_stream(ss.diag)
            if _BCAST_SA and q >= 3:
                grid.row_comm.bcast_sa(cb, root)
            else:
                grid.row_comm.bcast(cb, root)
            ev = ss.event(ss.diag)
        pend.append((a, b, cb, ev))
        nbytes = (b - a) * kb * esz
        st["row_msgs"] += 1
        st["row_bytes"] += nbytes
        if ci == 0:
            st["row_bytes_first"] = nbytes

    def land(i):
        a, b, cb, ev = pend[i]
        ss.wait(ss.panel, ev)
        if not own_col:
            Prow[a:b].copy_(cb)
    return Prow, land, (pend[0][2] if pend else Prow)


_GRAPHS = {}


class _SerialStreams:
    """StreamSet stand-in that keeps every step on the current stream."""
    gpu = True
    panel = diag = None
    update = [None]

    def use(self, st):
        import contextlib
        return contextlib.nullcontext()

    def wait(self, st, ev):
        pass

    def event(self, st=None):
        return None

    def fork(self, diag=True):
        pass

    def join(self):
        pass


def _potrf_graph_run(A, s, buf, nb, g0, nt, R_end, la, group, ss, ct, dev):
    """Option.UseGraph: the one-rank potrf captured once into a hipGraph per
    (buffer, geometry) and replayed -- one launch for the whole
    factorization, no host work per kernel: the form for launch-bound
    (small) orders, where the eager loop's ~30 launches per tile cost more
    than the kernels.  The capture records the single-stream form of the
    DAG: a capture that forks into the panel / update streams is not
    survived by this HIP runtime (hipStreamEndCapture segfaults on it,
    tools/probe/graph_probe2.py; a plain two-stream fork/join captures
    fine), so inside the graph the panel and the trailing update are
    ordered; large orders keep the eager pipelined path.  The info vector
    lives with the graph and is zeroed before each replay; replays read
    whatever A holds (same buffer)."""
    key = (buf.data_ptr(), buf.stride(1), g0, nt, nb, R_end, la, group, buf.dtype, str(dev))
    ent = _GRAPHS.get(key)
    if ent is None:
        infos = torch.zeros(max(nt, 1), dtype=torch.int64, device=dev)
        # warm-up on a scratch copy first: the launchers' per-stream
        # workspaces (csrc/hip/workspace.hpp) must exist for the capture
        # stream before the capture
        g = torch.cuda.CUDAGraph()
        # a PRIVATE stream, owned by the graph entry for its whole life: a
        # pooled torch stream can be handed to other code later, whose larger
        # workspace request on the same handle would free the buffers the
        # captured kernels point into (csrc/hip/workspace.hpp)
        from .. import _native
        cs = torch.cuda.ExternalStream(_native.hip().stream_create(dev.index if dev.index is not None
                                                                   else torch.cuda.current_device()),
                                       device=dev)
        cs.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(cs):
            scratch = buf.clone()
            _potrf_1x1_grouped(A, s, scratch, nb, g0, nt, R_end, la, group, ss, infos, ct, dev, serial=True)
            cs.synchronize()
            del scratch
            with torch.cuda.graph(g, stream=cs, capture_error_mode="relaxed"):
                _potrf_1x1_grouped(A, s, buf, nb, g0, nt, R_end, la, group, ss, infos, ct, dev, serial=True)
        torch.cuda.current_stream(dev).wait_stream(cs)
        ent = _GRAPHS[key] = (g, infos, cs)
    g, infos, _cs = ent
    infos.zero_()              # eagerly: a memset node inside the graph replays stale
    g.replay()
    return infos


def _potrf_info(s, infos, g0, nt):
    """First failing global column (1-based), reduced over ranks."""
    from ._util import read_to_host
    iv = read_to_host(infos).tolist()
    info = 0
    for t in range(nt):
        _wd.beat(f"potrf step {t}")
        if int(iv[t]) > 0:
            info = (s.row_offsets[g0 + t] - s.row_offsets[g0]) + int(iv[t])
            break
    if s.comm.size > 1:
        big = 1 << 62
        info = int(s.comm.allreduce_scalar(info if info > 0 else big, "min", torch.int64))
        info = 0 if info >= big else info
    return info


def _group_schedule(nt, G):
    """Tile groups of the one-rank potrf: G tiles per group (K = G nb
    trailing GEMMs), except the first SLATE_AMD_POTRF_HEAD and the last
    SLATE_AMD_POTRF_TAIL tiles, which go one per group.  At both ends the
    update stream idles behind the panel chain (kernel trace of the n =
    32768 bench, profiles/r6/potrf_1gpu_update_stream_gaps.txt: 2.6 ms idle
    in the first 10 % of the span, 7.0 ms in the last 10 %): a one-tile
    group halves that chain where the trailing GEMM is too small to hide it."""
    head = max(0, int(os.environ.get("SLATE_AMD_POTRF_HEAD", "0")))
    tail = max(0, int(os.environ.get("SLATE_AMD_POTRF_TAIL", "0")))
    head = min(head, nt)
    tail = min(tail, nt - head)
    out = [[t] for t in range(head)]
    out += [list(range(t, min(t + G, nt - tail))) for t in range(head, nt - tail, G)]
    out += [[t] for t in range(nt - tail, nt)]
    return out


def _potrf_1x1_grouped(A, s, buf, nb, g0, nt, R_end, la, G, ss, infos, ct, dev, serial=False):
    """One rank owning the whole matrix: panels are factored one tile at a
    time, but the trailing update is applied once per GROUP of G tiles with
    K = G nb (the G panel columns are adjacent in the local buffer, so the
    operand is a plain view): the MFMA GEMM runs at 61.8 TF/s with K = 1024
    against 58.5 at K = 512 (24576^2 NT, measured on MI355X).  Inside a
    group, tile u's column is brought up to date by the group's earlier
    panels (small GEMMs on the panel stream) right before its own panel.
    Lookahead counts groups: group g's panel stream also updates the next
    ``la`` groups' columns; the update stream does the rest, first the
    columns of group g + la + 1 (event), then everything else."""
    off = lambda t: s.row_offsets[min(g0 + t, g0 + nt)] if g0 + t < g0 + nt else R_end   # noqa: E731
    groups = _group_schedule(nt, G)
    ng = len(groups)
    gstart = lambda gi: off(groups[gi][0]) if gi < ng else R_end     # noqa: E731
    end = R_end

    def mask(r, c):
        return (1, nb, 1, 0, 1, 0, r, c, 0)

    def upd(P, c_lo, c_hi):
        """buf[c_lo:end, c_lo:c_hi] -= P[c_lo:, :] P[c_lo:c_hi, :]^H (lower mask);
        P's rows are indexed from its own first row ``P0``."""
        Pm, P0 = P
        if c_hi > c_lo:
            ops.gemm(-1.0, Pm[c_lo - P0:end - P0], Pm[c_lo - P0:c_hi - P0], 1.0, buf[c_lo:end, c_lo:c_hi], 'N', ct,
                     mask(c_lo, c_lo))

    ev_tr = {}
    if serial:
        ss = _SerialStreams()
    ss.fork(diag=False)
    for gi, tiles in enumerate(groups):
        _wd.beat(f"potrf group {gi}")
        c0, c2 = gstart(gi), gstart(gi + 1)
        with ss.use(ss.panel):
            if gi - la - 1 >= 0:
                ss.wait(ss.panel, ev_tr[gi - la - 1])
            with trace_block("potrf::panel"):
                for u in tiles:
                    cu, cu1 = off(u), off(u + 1)
                    if cu > c0:
                        # the group's earlier panels -> column u (rows >= cu)
                        upd((buf[c0:end, c0:cu], c0), cu, cu1)
                    ops.potrf('L', buf[cu:cu1, cu:cu1], infos[u:u + 1])
                    if end > cu1:
                        ops.trsm('R', 'L', ct, 'N', 1.0, buf[cu:cu1, cu:cu1], buf[cu1:end, cu:cu1])
            P = (buf[c0:end, c0:c2], c0)
            la_end = gstart(gi + 1 + la)
            if gi >= 1 and la > 0:
                ss.wait(ss.panel, ev_tr[gi - 1])
            upd(P, c2, la_end)
            ev_panel = ss.event(ss.panel)
        us = ss.update[0]
        with ss.use(us):
            ss.wait(us, ev_panel)
            nx_end = max(gstart(gi + 2 + la), la_end)
            with trace_block("potrf::trailing"):
                upd(P, la_end, nx_end)
                ev_tr[gi] = ss.event(us)
                upd(P, nx_end, end)
    ss.join()


def _lstart(g, nb, pr, p):
    from ..core.storage import local_start
    return local_start(g, nb, pr, p)


# ------------------------------------------------------------------ solves
def potrs(A, B, opts=None):
    """Solve A X = B with the Cholesky factor in A (lower or upper)."""
    from .blas3 import trsm
    if A.uplo() == Uplo.Lower:
        L = TriangularMatrix(Uplo.Lower, A, diag=Diag.NonUnit)
        trsm(Side.Left, 1.0, L, B, opts)
        trsm(Side.Left, 1.0, L.conj_transpose(), B, opts)
    else:
        U = TriangularMatrix(Uplo.Upper, A, diag=Diag.NonUnit)
        trsm(Side.Left, 1.0, U.conj_transpose(), B, opts)
        trsm(Side.Left, 1.0, U, B, opts)
    return 0


def posv(A, B, opts=None) -> int:
    from ..utils.timers import timer
    with timer("posv::potrf"):
        info = potrf(A, opts)
    if info == 0:
        with timer("posv::potrs"):
            potrs(A, B, opts)
    return info


def potri(A, opts=None) -> int:
    """Inverse from the Cholesky factor: A^{-1} = L^{-H} L^{-1} (trtri + trtrm)."""
    from .inverse import trtri, trtrm
    L = TriangularMatrix(A.uplo(), A, diag=Diag.NonUnit)
    info = trtri(L, opts)
    if info == 0:
        trtrm(L, opts)
    return info
