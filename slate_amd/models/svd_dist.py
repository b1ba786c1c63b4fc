"""Distributed SVD on a p x q process grid (no rank holds the dense matrix).

Reference: `src/svd.cc:155-364`, `src/ge2tb.cc` (column-panel QR and
row-panel LQ on the grid, two-sided trailing updates), `src/tb2bd.cc:54-200`
(band gathered to one rank, bulge chasing by host threads), `src/bdsqr.cc`
(every rank applies the rotations to its own rows of U / columns of V^H),
`src/unmbr_tb2bd.cc`, `src/unmbr_ge2tb.cc`.

MI355X design, per panel k of ``ge2tb_dist`` (A general m x n, m >= n, on a
copy with square tiles = the band width):

* column panel (tile column k, rows from tile k): all-gathered inside its
  process column and QR-factored there (deterministic kernels, so every
  rank of the column holds identical factors), written back in place
  (R on the band, reflectors below); V (this process row's rows) and T go
  along the process row in ONE packed broadcast;
* left update of the trailing columns: W = V^H C (local GEMM, summed over
  the process column), C -= V (T^H W);
* row panel (tile row k, columns from tile k+1): the transposed slab is
  all-gathered inside its process row and X^H is QR-factored there; X is
  written back as [L | V^H] (L on the band); V (rows = this process
  column's columns) and T go down the process column;
* right update of the rows below: Y = C V (local, summed over the process
  row), C -= (Y T) V^H.

The band (O(n nb) words) is reduced to rank 0, which runs the pipelined
host bulge chase (tb2bd); (d, e) and the chase reflectors are broadcast.
bdsqr runs on every rank on ITS rows of U and columns of V^H only (the
rotations depend on (d, e) alone, so all ranks make identical decisions).
The singular vectors then move P x 1 -> 1 x P (piece-level redistribution)
for the chase reflectors, and onto the grid of the stage-1 factors: U on
A's grid, V on the TRANSPOSED grid (its rows distributed like A's
columns, so the row-panel reflectors apply without any data movement).
"""
from __future__ import annotations

import torch

from .. import _native, ops
from ..core.enums import GridOrder, Norm, Option, Uplo
from ..core.exceptions import SlateError
from ..core.options import get_option
from ..core.storage import numroc
from ..utils.trace import trace_block
from ._panels import panel_allgather
from .eig_dist import _bcast_dev, _bcast_host   # O(n) vectors via host, the reflectors device to device
from ._util import conj_trans, grid_of, target_slot, tiles_local_before


class Ge2tbDistFactors:
    """left: (k, kk, T) -- V in tile column k from tile row k;
    right: (k, kr, T) -- V^H in tile row k from tile column k + 1."""

    def __init__(self, nb):
        self.nb = nb
        self.left = []
        self.right = []


def _general(like, m, n, nb, p, q, order):
    from ..core.matrix import Matrix
    s = like.storage
    M = Matrix(m, n, nb=nb, p=p, q=q, comm=s.comm, dtype=s.dtype, device=s.device, order=order)
    M.insertLocalTiles(device=s.device.index if s.device.type == "cuda" else -1)
    return M


def _flip(order):
    return GridOrder.Row if order == GridOrder.Col else GridOrder.Col


def ge2tb_dist(G, opts=None):
    """Reduce the general block-cyclic G (m >= n, square tiles) in place to
    upper band form (bandwidth = tile size); returns the panel factors."""
    s = G.storage
    bc = s.bc
    grid = grid_of(G)
    nb, p, q, pr, pc = bc.nb, bc.p, bc.q, bc.pr, bc.pc
    m, n = G.m(), G.n()
    if m < n:
        raise SlateError("ge2tb_dist: needs m >= n (factor the conjugate transpose)")
    nt = G.nt()
    buf = s.prepare_local(target_slot(G, opts))
    dev, dt = buf.device, s.dtype
    ct = conj_trans(dt)
    mloc, nloc = bc.mloc, bc.nloc
    mloc_r = [numroc(m, nb, r, p) for r in range(p)]
    nloc_c = [numroc(n, nb, c, q) for c in range(q)]
    Fac = Ge2tbDistFactors(nb)
    from .lu import _Pack
    with trace_block("ge2tb"):
        for k in range(nt):
            c0 = k * nb
            kb = min(nb, n - c0)
            kk = min(m - c0, kb)
            ck, rk = k % q, k % p
            lr_k = min(tiles_local_before(k, p, pr) * nb, mloc)
            lr1 = min(tiles_local_before(k + 1, p, pr) * nb, mloc)
            lc_k = min(tiles_local_before(k, q, pc) * nb, nloc)
            lc1 = min(tiles_local_before(k + 1, q, pc) * nb, nloc)
            nmine = mloc - lr_k
            # ---- column panel QR
            pk = _Pack([("T", kk, kk, dt), ("V", nmine, kk, dt)], dev)
            Tk, Vloc = pk.get("T"), pk.get("V")
            with trace_block("ge2tb::qr"):
                if pc == ck:
                    P, myidx = panel_allgather(grid.col_comm if grid else None, buf, mloc, k, lc_k, kb, nb, p, pr,
                                               mloc_r, dt, dev)
                    tau = torch.zeros(kk, dtype=dt, device=dev)
                    Vf = ops.colmajor_empty(m - c0, kk, dt, dev)
                    ops.geqrf(P, tau, Tk, Vf)
                    if nmine:
                        ops.row_gather(P, buf[lr_k:mloc, lc_k:lc_k + kb], myidx)
                        ops.row_gather(Vf, Vloc, myidx)
                if q > 1:
                    grid.row_comm.bcast(pk.raw, ck)
            Fac.left.append((k, kk, Tk.clone()))
            C = buf[lr_k:mloc, lc1:nloc]
            if C.shape[1]:
                W = ops.colmajor_zeros(kk, C.shape[1], dt, dev)
                if nmine:
                    ops.gemm(1.0, Vloc, C, 0.0, W, transA=ct)                  # V^H C (partial)
                if p > 1:
                    grid.col_comm.allreduce(W)
                ops.trmm('L', 'U', ct, 'N', 1.0, Tk, W)                       # T^H V^H C
                if nmine:
                    ops.gemm(-1.0, Vloc, W, 1.0, C)
            if k + 1 >= nt:
                continue
            # ---- row panel LQ (QR of X^H)
            w = n - (c0 + kb)
            kr = min(w, kb)
            ncl = nloc - lc1
            pk2 = _Pack([("T", kr, kr, dt), ("V", ncl, kr, dt)], dev)
            Tr, Vr = pk2.get("T"), pk2.get("V")
            with trace_block("ge2tb::lq"):
                if pr == rk:
                    S = ops.colmajor_empty(nloc, kb, dt, dev)            # rows = local columns
                    if nloc:
                        S.copy_(buf[lr_k:lr_k + kb, :nloc].mT)
                    Pt, myc = panel_allgather(grid.row_comm if grid else None, S, nloc, k + 1, 0, kb, nb, q, pc,
                                              nloc_c, dt, dev)              # X^T, global column order
                    if dt.is_complex:
                        Xh = ops.colmajor_empty(w, kb, dt, dev)
                        Xh.copy_(Pt.conj())
                    else:
                        Xh = Pt
                    taur = torch.zeros(kr, dtype=dt, device=dev)
                    Vrf = ops.colmajor_empty(w, kr, dt, dev)
                    ops.geqrf(Xh, taur, Tr, Vrf)
                    if ncl:
                        tmp = ops.colmajor_empty(ncl, kb, dt, dev)
                        ops.row_gather(Xh, tmp, myc)
                        buf[lr_k:lr_k + kb, lc1:nloc].copy_(tmp.mH)      # [L | V^H]
                        ops.row_gather(Vrf, Vr, myc)
                if p > 1:
                    grid.col_comm.bcast(pk2.raw, rk)
            Fac.right.append((k, kr, Tr.clone()))
            C2 = buf[lr1:mloc, lc1:nloc]
            if C2.shape[0]:
                Y = ops.colmajor_zeros(C2.shape[0], kr, dt, dev)
                if ncl:
                    ops.gemm(1.0, C2, Vr, 0.0, Y)                            # C V (partial)
                if q > 1:
                    grid.row_comm.allreduce(Y)
                ops.trmm('R', 'U', 'N', 'N', 1.0, Tr, Y)                    # C V T
                if ncl:
                    ops.gemm(-1.0, Y, Vr, 1.0, C2, transB=ct)
    s.mark_local_modified(s.origin_slot)
    return Fac


def gather_upper_band(G, root=0):
    """Upper band of the reduced G (upper triangles of the diagonal tiles,
    lower triangles of the super-diagonal tiles) as a dense host n x n
    matrix on ``root`` (None elsewhere); one (2 nb) x n sum-reduction."""
    s = G.storage
    bc = s.bc
    nb, p, q, pr, pc = bc.nb, bc.p, bc.q, bc.pr, bc.pc
    n, nt = G.n(), G.nt()
    buf = s.local[s.origin_slot]
    dev, dt = buf.device, s.dtype
    stack = ops.colmajor_zeros(2 * nb, max(n, 1), dt, dev)
    for j in range(nt):
        c0 = j * nb
        kb = min(nb, n - c0)
        if j % q != pc:
            continue
        lc = tiles_local_before(j, q, pc) * nb
        if j >= 1 and (j - 1) % p == pr:
            lr = tiles_local_before(j - 1, p, pr) * nb
            ops.gecopy(buf[lr:lr + nb, lc:lc + kb], stack[0:nb, c0:c0 + kb], uplo='L')
        if j % p == pr:
            lr = tiles_local_before(j, p, pr) * nb
            ops.gecopy(buf[lr:lr + kb, lc:lc + kb], stack[nb:nb + kb, c0:c0 + kb], uplo='U')
    comm = s.comm
    if comm.size > 1:
        comm.reduce(stack, root)
    if comm.rank != root:
        return None
    # assembled on the root's device by masked copies (no host n x n)
    B = ops.colmajor_zeros(n, n, dt, dev)
    for j in range(nt):
        c0 = j * nb
        kb = min(nb, n - c0)
        ops.gecopy(stack[nb:nb + kb, c0:c0 + kb], B[c0:c0 + kb, c0:c0 + kb], uplo='U')
        if j >= 1:
            ops.gecopy(stack[0:nb, c0:c0 + kb], B[c0 - nb:c0, c0:c0 + kb], uplo='L')
    return B


def _apply_left(G, Fac, Z):
    """Z := Q Z, Q = H_0 H_1 ... (column-panel reflectors of G); Z shares
    G's row distribution."""
    sG, sZ = G.storage, Z.storage
    bc = sG.bc
    grid = grid_of(G)
    nb, p, q, pr, pc = bc.nb, bc.p, bc.q, bc.pr, bc.pc
    mloc = bc.mloc
    gbuf = sG.local[sG.origin_slot]
    zbuf = Z.local_block().data
    dev, dt = gbuf.device, sG.dtype
    ct = conj_trans(dt)
    for (k, kk, Tk) in reversed(Fac.left):
        lr0 = min(tiles_local_before(k, p, pr) * nb, mloc)
        lc_k = tiles_local_before(k, q, pc) * nb
        nmine = mloc - lr0
        V = ops.colmajor_empty(nmine, kk, dt, dev)
        if pc == k % q and nmine:
            src = gbuf[lr0:mloc, lc_k:lc_k + kk]
            if pr == k % p:
                ops.v_explicit(src, V)
            else:
                V.copy_(src)
        if q > 1:
            from ..parallel.tilecomm import bcast_tile
            bcast_tile(grid.row_comm, V, k % q)
        C = zbuf[lr0:mloc, :]
        if not C.shape[1]:
            continue
        W = ops.colmajor_zeros(kk, C.shape[1], dt, dev)
        if nmine:
            ops.gemm(1.0, V, C, 0.0, W, transA=ct)
        if p > 1:
            grid.col_comm.allreduce(W)
        ops.trmm('L', 'U', 'N', 'N', 1.0, Tk, W)
        if nmine:
            ops.gemm(-1.0, V, W, 1.0, C)
    sZ.mark_local_modified(sZ.origin_slot)


def _apply_right(G, Fac, Zt):
    """Zt := P Zt, P = G_0 G_1 ... (row-panel reflectors of G); Zt (n x k)
    lives on the TRANSPOSED grid: its local rows are G's local columns."""
    sG, sZ = G.storage, Zt.storage
    bc = sG.bc
    grid = grid_of(G)
    nb, p, q, pr, pc = bc.nb, bc.p, bc.q, bc.pr, bc.pc
    nloc = bc.nloc
    gbuf = sG.local[sG.origin_slot]
    zbuf = Zt.local_block().data
    dev, dt = gbuf.device, sG.dtype
    ct = conj_trans(dt)
    for (k, kr, Tr) in reversed(Fac.right):
        lr_k = tiles_local_before(k, p, pr) * nb
        lc1 = min(tiles_local_before(k + 1, q, pc) * nb, nloc)
        ncl = nloc - lc1
        V = ops.colmajor_empty(ncl, kr, dt, dev)
        if pr == k % p and ncl:
            tmp = ops.colmajor_empty(ncl, kr, dt, dev)
            tmp.copy_(gbuf[lr_k:lr_k + kr, lc1:nloc].mH)
            if pc == (k + 1) % q:
                ops.v_explicit(tmp, V)
            else:
                V.copy_(tmp)
        if p > 1:
            from ..parallel.tilecomm import bcast_tile
            bcast_tile(grid.col_comm, V, k % p)
        C = zbuf[lc1:nloc, :]
        if not C.shape[1]:
            continue
        W = ops.colmajor_zeros(kr, C.shape[1], dt, dev)
        if ncl:
            ops.gemm(1.0, V, C, 0.0, W, transA=ct)
        if q > 1:
            grid.row_comm.allreduce(W)
        ops.trmm('L', 'U', 'N', 'N', 1.0, Tr, W)
        if ncl:
            ops.gemm(-1.0, V, W, 1.0, C)
    sZ.mark_local_modified(sZ.origin_slot)




def svd_dist(A, S=None, U=None, VH=None, opts=None):
    """Distributed svd (see module docstring).  Returns the singular values
    (host fp64, descending) on every rank; fills U (m x k) / VH (k x n),
    k = min(m, n), when given.  A is not modified (stage 1 runs on a copy)."""
    from . import svd as SV
    from .aux import copy, copy_conj_transpose, norm, redistribute, scale as mscale, set as aset
    from .eig import Hb2stFactors
    s = A.storage
    comm = s.comm
    P = comm.size
    m, n = A.m(), A.n()
    bcA = s.bc
    with trace_block("svd"):
        band = int(get_option(opts, Option.InnerBlocking, 0) or 0) or min(bcA.nb, 64)
        trans = m < n
        if trans:
            G = _general(A, n, m, band, bcA.p, bcA.q, bcA.order)
            copy_conj_transpose(A, G)
            m, n = n, m
            U, VH = VH, U          # A^H = Ug S Vg^H  ->  U = Vg, VH = Ug^H
        else:
            G = _general(A, m, n, band, bcA.p, bcA.q, bcA.order)
            copy(A, G)
        k = n
        amax = float(norm(Norm.Max, G))
        sc = 1.0
        if amax > 0 and (amax < 1e-140 or amax > 1e140):
            sc = 1.0 / amax
            mscale(sc, 1.0, G)
        Fac = ge2tb_dist(G, opts)
        B = gather_upper_band(G, root=0)
        wantU, wantV = U is not None, VH is not None
        dt = s.dtype
        if comm.rank == 0:
            d, e, F2 = SV.tb2bd(B, band)
            meta = torch.tensor([F2.U.count, F2.V.count], dtype=torch.int64)
        else:
            d = e = F2 = None
            meta = torch.zeros(2, dtype=torch.int64)
        meta = _bcast_host(comm, meta, 0)
        d = _bcast_host(comm, d if d is not None else torch.zeros(k, dtype=torch.float64), 0)
        e = _bcast_host(comm, e if e is not None else torch.zeros(max(k - 1, 0), dtype=torch.float64), 0)
        if not (wantU or wantV):
            sv, _, _ = SV.bdsqr(d, e, False, False)
        else:
            dev = G.storage.local[G.storage.origin_slot].device
            parts = []
            for which, cnt in (("U", int(meta[0])), ("V", int(meta[1]))):
                if comm.rank == 0:
                    F = getattr(F2, which)
                    t = (F.V, F.tau, F.row, F.length, F.sweep_ptr)
                else:
                    t = (torch.zeros(cnt, band, dtype=dt, device=dev), torch.zeros(cnt, dtype=dt, device=dev),
                         torch.zeros(cnt, dtype=torch.int64, device=dev),
                         torch.zeros(cnt, dtype=torch.int64, device=dev),
                         torch.zeros(max(k, 1), dtype=torch.int64, device=dev))
                t = tuple(_bcast_dev(comm, x, 0, dev) for x in t)
                parts.append(Hb2stFactors(t[0], t[1], t[2], t[3], t[4], cnt, None))
            FU, FV = parts
            pu = _bcast_host(comm, F2.pu if comm.rank == 0 else torch.ones(k, dtype=dt), 0)
            pv = _bcast_host(comm, F2.pv if comm.rank == 0 else torch.ones(k, dtype=dt), 0)
            # bdsqr on this rank's rows of U / columns of V^H (a P x 1 layout)
            Lu = _general(G, k, k, band, P, 1, GridOrder.Col)
            lb = Lu.local_block()
            rows = torch.as_tensor([lb.global_row(i) for i in range(lb.mloc)], dtype=torch.int64)
            nr = rows.numel()
            eye = torch.eye(k, dtype=torch.float64)
            Uh = eye[rows, :].t().contiguous().t() if (wantU and nr) else None       # nr x k
            VTh = eye[:, rows].t().contiguous().t() if (wantV and nr) else None      # k x nr
            dd = d.to(torch.float64).clone()
            ee = e.to(torch.float64).clone() if k > 1 else torch.zeros(1, dtype=torch.float64)
            with trace_block("bdsqr"):
                f = _native._host.bdsqr(k, dd.data_ptr(), ee.data_ptr(),
                                        Uh.data_ptr() if Uh is not None else 0, max(1, nr),
                                        nr if Uh is not None else 0,
                                        VTh.data_ptr() if VTh is not None else 0, max(1, k),
                                        nr if VTh is not None else 0)
            if f:
                raise SlateError("bdsqr: no convergence")
            sv = dd
            Zouts = {}
            for which, want, Hm, ph, F2x in (("U", wantU, Uh, pu, FU), ("V", wantV, VTh, pv, FV)):
                if not want:
                    continue
                # full height (U: m rows, zero below k), P x 1: this rank's
                # rows < k are its first local rows (block-cyclic keeps order)
                mr = m if which == "U" else k
                Zp = _general(G, mr, k, band, P, 1, GridOrder.Col)
                aset(0.0, 0.0, Zp)
                zl = Zp.local_block()
                if nr:
                    blk = Hm if which == "U" else Hm.t()                           # nr x k
                    zl.data[:nr, :k].copy_((ph[rows][:, None] * blk.to(dt)).to(dev))
                Zp.storage.mark_local_modified(Zp.storage.origin_slot)
                Z1 = _general(G, mr, k, band, 1, P, GridOrder.Col)
                redistribute(Zp, Z1)
                lb1 = Z1.local_block()
                if lb1.nloc:
                    Zl = ops.colmajor_empty(k, lb1.nloc, dt, dev)
                    Zl.copy_(lb1.data[:k, :lb1.nloc])
                    SV._unmtr_refl(F2x, Zl)
                    lb1.data[:k, :lb1.nloc].copy_(Zl)
                Z1.storage.mark_local_modified(Z1.storage.origin_slot)
                bg = G.storage.bc
                if which == "U":
                    Zg = _general(G, m, k, band, bg.p, bg.q, bg.order)
                    redistribute(Z1, Zg)
                    _apply_left(G, Fac, Zg)
                else:
                    Zg = _general(G, k, k, band, bg.q, bg.p, _flip(bg.order))
                    redistribute(Z1, Zg)
                    _apply_right(G, Fac, Zg)
                Zouts[which] = Zg
            if wantU:
                Zu = Zouts["U"]
                if trans:
                    copy_conj_transpose(Zu, U)      # caller's VH = Ug^H
                else:
                    redistribute(Zu, U)
            if wantV:
                Zv = Zouts["V"]
                if trans:
                    redistribute(Zv, VH)            # caller's U = Vg
                else:
                    copy_conj_transpose(Zv, VH)
        if sc != 1.0:
            sv = sv / sc
        if S is not None:
            S.copy_(sv.to(S.dtype).to(S.device)[:S.numel()])
        return sv
