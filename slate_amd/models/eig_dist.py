"""Distributed two-stage Hermitian eigensolver on a p x q process grid.

Reference: `src/heev.cc:66-225`, `src/he2hb.cc:26-677` (panel QR + two-sided
trailing update on the grid), `src/hb2st.cc:139-279` (band gathered to one
rank, bulge chasing by host threads), `src/stedc*.cc`,
`src/unmtr_hb2st.cc`, `src/unmtr_he2hb.cc`.

MI355X design (no rank ever holds the dense matrix):

* stage 1, ``he2hb_dist``: the trailing matrix is kept with BOTH triangles
  (a general block-cyclic copy -- HBM is plentiful, and Y = A V T becomes
  one local GEMM per rank instead of a symmetric-storage hemm with a
  transposed-contribution reduction).  Per panel k:
    - the panel (tile column k, rows from tile k+1) is all-gathered inside
      its process column and QR-factored there by every rank redundantly
      (deterministic kernels), the factored rows written back in place
      (R in tile (k+1, k), reflectors below: SLATE layout);
    - V and T travel along the process rows in ONE packed broadcast;
    - X = V T; the rows of X (later W, V) indexed by this rank's local
      COLUMNS are assembled by column broadcasts (`_panels.assemble_cols`);
    - Y = A22 X: one local GEMM, summed over the process row (all-reduce);
    - M = X^H Y: local GEMM, summed over the process column (kb x kb);
    - W = Y - V M / 2;  A22 -= V W^H + W V^H: two local GEMMs.
* the band (tile diagonal + R blocks, O(n nb) words) is reduced to rank 0,
  which runs the pipelined multi-threaded bulge chase (`_host.hb2st`) and
  broadcasts (d, e) and the reflectors;
* the tridiagonal eigenproblem is solved on every rank (GPU merges);
* back-transforms: each rank applies Q2 (bulge reflectors) to ITS columns
  of Z (a 1 x P column-cyclic layout, full height), Z is redistributed to
  the caller's grid (piece-level exchange), and Q1 is applied on the grid
  with the panel reflectors read back from the factored matrix (row
  broadcast per panel, V^H Z summed over the process column).
"""
from __future__ import annotations

import torch

from .. import ops
from ..core.enums import Uplo
from ..core.exceptions import SlateError
from ..core.storage import numroc
from ..utils.trace import trace_block
from ._panels import assemble_cols, panel_allgather, plan_col_gather
from ._util import conj_trans, grid_of, target_slot, tiles_local_before


def _new_general(A, m=None, n=None, p=None, q=None, nb=None):
    from ..core.matrix import Matrix
    s = A.storage
    bc = s.bc
    M = Matrix(m if m is not None else A.m(), n if n is not None else A.n(), nb=nb or bc.nb,
               p=p or bc.p, q=q or bc.q, comm=s.comm, dtype=s.dtype, device=s.device, order=bc.order)
    M.insertLocalTiles(device=s.device.index if s.device.type == "cuda" else -1)
    return M


def full_hermitian_copy(A, nb=None):
    """General block-cyclic copy of Hermitian A holding both triangles, with
    tile size nb (default A's) -- piece-level redistribution of the stored
    triangle and its conjugate transpose; no gather."""
    from .aux import copy, copy_conj_transpose, set as aset, set_diag_imag_zero
    from ..core.matrix import TriangularMatrix as TM
    F = _new_general(A, nb=nb)
    aset(0.0, 0.0, F)
    up = A.uploPhysical()
    stored = TM(up, A)
    if up == Uplo.Lower:
        copy(stored, TM(Uplo.Lower, F))
        copy_conj_transpose(stored, TM(Uplo.Upper, F))
    else:
        copy(stored, TM(Uplo.Upper, F))
        copy_conj_transpose(stored, TM(Uplo.Lower, F))
    if F.storage.dtype.is_complex:
        set_diag_imag_zero(F)
    return F


class He2hbDistFactors:
    """Per panel: (k, r0, kk, T) -- V stays in the factored matrix."""

    def __init__(self, nb):
        self.nb = nb
        self.panels = []


def he2hb_dist(F, opts=None):
    """Reduce the full Hermitian block-cyclic F in place to band form
    (bandwidth nb = tile size); returns the panel factors."""
    s = F.storage
    bc = s.bc
    grid = grid_of(F)
    nb, p, q, pr, pc = bc.nb, bc.p, bc.q, bc.pr, bc.pc
    n = F.n()
    nt = F.nt()
    slot = target_slot(F, opts)
    buf = s.prepare_local(slot)
    dev, dt = buf.device, s.dtype
    ct = conj_trans(dt)
    mloc, nloc = bc.mloc, bc.nloc
    nloc_r = [numroc(n, nb, r, p) for r in range(p)]
    Fac = He2hbDistFactors(nb)
    from .lu import _Pack
    from ..parallel.streams import StreamSet
    # lookahead (src/he2hb.cc:172-610): the rank-2k update of step k first
    # touches the next panel's tile column (event), then the rest; panel
    # k+1 (all-gather, QR, broadcast) runs on the high-priority panel stream
    # as soon as that column is done, concurrently with step k's bulk GEMMs
    ss = StreamSet(dev, reserve_cus=0)
    us = ss.update[0]
    ev_la = {}
    ss.fork(diag=False)
    with trace_block("he2hb"):
        for k in range(nt - 1):
            r0 = (k + 1) * nb
            kb = min(nb, n - k * nb)
            m2 = n - r0
            kk = min(m2, kb)
            ck = k % q
            lr0 = min(tiles_local_before(k + 1, p, pr) * nb, mloc)
            lc_k = min(tiles_local_before(k, q, pc) * nb, nloc)
            lc1 = min(tiles_local_before(k + 1, q, pc) * nb, nloc)
            lc2 = min(tiles_local_before(k + 2, q, pc) * nb, nloc)
            nmine = mloc - lr0
            with ss.use(ss.panel):
                if k >= 1:
                    ss.wait(ss.panel, ev_la[k - 1])
                pk = _Pack([("T", kk, kk, dt), ("V", nmine, kk, dt)], dev)
                Tk, Vloc = pk.get("T"), pk.get("V")
                with trace_block("he2hb::panel"):
                    if pc == ck:
                        P, myidx = panel_allgather(grid.col_comm, buf, mloc, k + 1, lc_k, kb, nb, p, pr, nloc_r,
                                                   dt, dev)
                        tau = torch.zeros(kk, dtype=dt, device=dev)
                        Vf = ops.colmajor_empty(m2, kk, dt, dev)
                        ops.geqrf(P, tau, Tk, Vf)
                        if nmine:
                            ops.row_gather(P, buf[lr0:mloc, lc_k:lc_k + kb], myidx)
                            ops.row_gather(Vf, Vloc, myidx)
                    if q > 1:
                        grid.row_comm.bcast(pk.raw, ck)
                Fac.panels.append((k, r0, kk, pk.prefix("V").get("T")))
                ev_panel = ss.event(ss.panel)
            with ss.use(us):
                ss.wait(us, ev_panel)
                if buf.is_cuda:
                    pk.raw.record_stream(us)
                with trace_block("he2hb::update"):
                    plan = plan_col_gather(s.tileMb, k + 1, nt, nb, p, q, pc, dev)
                    X = ops.colmajor_empty(nmine, kk, dt, dev)
                    if nmine:
                        X.copy_(Vloc)
                        ops.trmm('R', 'U', 'N', 'N', 1.0, Tk, X)                      # X = V T
                    Xc = assemble_cols(plan, X, grid, p, kk, dt, dev)
                    A22 = buf[lr0:mloc, lc1:nloc]
                    Y = ops.colmajor_zeros(nmine, kk, dt, dev)
                    if nmine and A22.shape[1]:
                        ops.gemm(1.0, A22, Xc, 0.0, Y)                                 # partial A V T
                    if q > 1 and nmine:
                        grid.row_comm.allreduce(Y)
                    M = ops.colmajor_zeros(kk, kk, dt, dev)
                    if nmine:
                        ops.gemm(1.0, X, Y, 0.0, M, transA=ct)                         # partial T^H V^H Y
                    if p > 1:
                        grid.col_comm.allreduce(M)
                    if nmine:
                        ops.gemm(-0.5, Vloc, M, 1.0, Y)                                # W = Y - V M / 2
                    Wc = assemble_cols(plan, Y, grid, p, kk, dt, dev)
                    Vc = assemble_cols(plan, Vloc, grid, p, kk, dt, dev)
                    for (a, b) in ((lc1, lc2), (lc2, nloc)):
                        if nmine and b > a:
                            Ab = buf[lr0:mloc, a:b]
                            ops.gemm(-1.0, Vloc, Wc[a - lc1:b - lc1], 1.0, Ab, transB=ct)   # A -= V W^H
                            ops.gemm(-1.0, Y, Vc[a - lc1:b - lc1], 1.0, Ab, transB=ct)      # A -= W V^H
                        if a == lc1:
                            ev_la[k] = ss.event(us)
    ss.join()
    s.mark_local_modified(slot)
    return Fac


def gather_band(F, root=0):
    """The Hermitian band of the reduced F (tile diagonal, lower triangle +
    the R blocks of the sub-diagonal tiles) as a dense n x n matrix on
    ``root``'s device (both triangles; None elsewhere), the stage-2 chase's
    input.  Each rank contributes the band tiles it owns to a (2 nb) x n
    stack; one sum-reduction, O(n nb) traffic.  The root assembles it with
    kernels on the device -- no host n x n (SLATE he2hbGather,
    HermitianBandMatrix.hh:310, gathers into band storage; the GPU chase
    works on a dense window of the band)."""
    s = F.storage
    bc = s.bc
    nb, p, q, pr, pc = bc.nb, bc.p, bc.q, bc.pr, bc.pc
    n, nt = F.n(), F.nt()
    buf = s.local[s.origin_slot]
    dev, dt = buf.device, s.dtype
    stack = ops.colmajor_zeros(2 * nb, max(n, 1), dt, dev)
    for k in range(nt):
        c0 = k * nb
        kb = min(nb, n - c0)
        if k % q != pc:
            continue
        lc = tiles_local_before(k, q, pc) * nb
        if k % p == pr:
            lr = tiles_local_before(k, p, pr) * nb
            ops.gecopy(buf[lr:lr + kb, lc:lc + kb], stack[0:kb, c0:c0 + kb], uplo='L')
        if k + 1 < nt and (k + 1) % p == pr:
            lr = tiles_local_before(k + 1, p, pr) * nb
            kr = min(nb, n - (k + 1) * nb)
            ops.gecopy(buf[lr:lr + kr, lc:lc + kb], stack[nb:nb + kr, c0:c0 + kb], uplo='U')
    comm = s.comm
    if comm.size > 1:
        comm.reduce(stack, root)
    if comm.rank != root:
        return None
    big = 1 << 40
    lower = (1, big, 1, 0, 1, 0, 0, 0, 0)         # row >= col (TriMask tuple)
    supper = (2, big, 1, 0, 1, 0, 0, 0, -1)       # row < col
    B = ops.colmajor_zeros(n, n, dt, dev)
    for k in range(nt):
        c0 = k * nb
        kb = min(nb, n - c0)
        ops.gecopy_mask(stack[0:kb, c0:c0 + kb], B[c0:c0 + kb, c0:c0 + kb], lower, real_diag=True)
        if k + 1 < nt:
            kr = min(nb, n - (k + 1) * nb)
            ops.gecopy(stack[nb:nb + kr, c0:c0 + kb], B[c0 + nb:c0 + nb + kr, c0:c0 + kb], uplo='U')
    # the upper triangle: the strictly lower band conjugate-transposed
    Bt = ops.colmajor_empty(n, n, dt, dev)
    ops.gecopy(B, Bt, trans=conj_trans(dt))
    ops.gecopy_mask(Bt, Bt, supper)
    ops.geadd(1.0, Bt, 1.0, B)
    return B


def unmtr_he2hb_dist(F, Fac: He2hbDistFactors, Z):
    """Z := Q1 Z on the grid (Q1 = H_0 H_1 ..., panels last to first); Z has
    F's row distribution.  V of panel k is read from the factored F on the
    panel's process column and broadcast along the process rows."""
    sF, sZ = F.storage, Z.storage
    bc, bz = sF.bc, sZ.bc
    if (bz.p, bz.pr, bz.mb) != (bc.p, bc.pr, bc.mb) or Z.global_offsets() != (0, 0):
        raise SlateError("unmtr_he2hb_dist: Z must share F's row distribution")
    grid = grid_of(F)
    nb, p, q, pr, pc = bc.nb, bc.p, bc.q, bc.pr, bc.pc
    mloc = bc.mloc
    fbuf = sF.local[sF.origin_slot]
    zl = Z.local_block()
    zbuf = zl.data
    dev, dt = fbuf.device, sF.dtype
    ct = conj_trans(dt)
    with trace_block("unmtr_he2hb"):
        for (k, r0, kk, Tk) in reversed(Fac.panels):
            lr0 = min(tiles_local_before(k + 1, p, pr) * nb, mloc)
            lc_k = tiles_local_before(k, q, pc) * nb
            nmine = mloc - lr0
            V = ops.colmajor_empty(nmine, kk, dt, dev)
            if pc == k % q and nmine:
                src = fbuf[lr0:mloc, lc_k:lc_k + kk]
                if pr == (k + 1) % p:
                    ops.v_explicit(src, V)          # the panel's first rows: unit lower
                else:
                    V.copy_(src)
            if q > 1:
                from ..parallel.tilecomm import bcast_tile
                bcast_tile(grid.row_comm, V, k % q)
            C = zbuf[lr0:mloc, :]
            W = ops.colmajor_zeros(kk, C.shape[1], dt, dev)
            if nmine and C.shape[1]:
                ops.gemm(1.0, V, C, 0.0, W, transA=ct)
            if p > 1 and C.shape[1]:
                grid.col_comm.allreduce(W)
            if C.shape[1]:
                ops.trmm('L', 'U', 'N', 'N', 1.0, Tk, W)
                if nmine:
                    ops.gemm(-1.0, V, W, 1.0, C)
    sZ.mark_local_modified(sZ.origin_slot)
    return Z


def heev_dist(A, Lambda=None, Z=None, opts=None):
    """Distributed heev (see module docstring).  Returns the eigenvalues
    (host fp64, ascending) on every rank; fills Z when given."""
    from . import eig as E
    from .aux import norm, redistribute, scale as mscale
    from ..core.enums import MethodEig, Norm, Option
    from ..core.options import get_option
    s = A.storage
    comm = s.comm
    n = A.n()
    with trace_block("heev"):
        # stage-1 band = F's tile size: InnerBlocking, default min(nb, 64)
        band = int(get_option(opts, Option.InnerBlocking, 0) or 0) or min(s.bc.nb, 64)
        F = full_hermitian_copy(A, nb=band)
        dev = F.storage.local[F.storage.origin_slot].device
        amax = float(norm(Norm.Max, F))
        sc = 1.0
        if amax > 0 and (amax < 1e-140 or amax > 1e140):
            sc = 1.0 / amax
            mscale(sc, 1.0, F)
        Fac = he2hb_dist(F, opts)
        nb = F.storage.bc.nb
        B = gather_band(F, root=0)
        want = Z is not None
        method = get_option(opts, Option.MethodEig, MethodEig.DC)
        # stage 2 on rank 0, results broadcast
        if comm.rank == 0:
            d, e, F2 = E.hb2st(B, nb, device=dev if dev.type == "cuda" else None)
            meta = torch.tensor([F2.count], dtype=torch.int64)
        else:
            d = e = F2 = None
            meta = torch.zeros(1, dtype=torch.int64)
        meta = _bcast_host(comm, meta, 0)
        cnt = int(meta[0])
        d = _bcast_host(comm, d if d is not None else torch.zeros(n, dtype=torch.float64), 0)
        e = _bcast_host(comm, e if e is not None else torch.zeros(max(n - 1, 0), dtype=torch.float64), 0)
        if not want:
            w = E.sterf(d, e)
        else:
            dt = s.dtype
            # the reflectors (~n^2/2 words) go device to device over the
            # communicator; only O(n) vectors take the host path above
            if comm.rank == 0:
                parts = (F2.V, F2.tau, F2.row, F2.length, F2.sweep_ptr, F2.phase)
            else:
                parts = (torch.zeros(cnt, nb, dtype=dt, device=dev), torch.zeros(cnt, dtype=dt, device=dev),
                         torch.zeros(cnt, dtype=torch.int64, device=dev),
                         torch.zeros(cnt, dtype=torch.int64, device=dev),
                         torch.zeros(max(n, 1), dtype=torch.int64, device=dev), torch.ones(n, dtype=dt, device=dev))
            parts = tuple(_bcast_dev(comm, t, 0, dev) for t in parts)
            F2 = E.Hb2stFactors(parts[0], parts[1], parts[2], parts[3], parts[4], cnt, parts[5])
            # Q2 on this rank's columns of a 1 x P column-cyclic Z, then onto Z's grid
            P = comm.size
            Z1 = _new_general(Z, n, n, 1, P, nb) if P > 1 else None
            Zc = Z1 if Z1 is not None else Z
            lb = Zc.local_block()
            if P > 1 and method not in (MethodEig.QR, 'Q', "qr"):
                # distributed D&C: the tridiagonal eigenvectors stay
                # row-distributed (no n x n on any rank, models/stedc.py),
                # then ONE redistribution to the column-cyclic layout the
                # back-transform runs on
                from .stedc import stedc_matrix
                w, Zr = stedc_matrix(d.numpy(), e.numpy(), comm, dev, nb, dtype=dt)
                redistribute(Zr, Z1)
                del Zr
                if lb.nloc:
                    Zl = lb.data[:n, :lb.nloc]
                    E.unmtr_hb2st(F2, Zl)
            else:
                if method in (MethodEig.QR, 'Q', "qr"):
                    w, Zt = E.steqr(d, e)
                else:
                    w, Zt = E.stedc(d, e, device=dev)
                cols = [lb.global_col(j) for j in range(lb.nloc)]
                if cols:
                    idx = torch.as_tensor(cols, device=Zt.device)
                    Zl = ops.as_colmajor(Zt[:, idx].to(dt).to(dev).contiguous())
                    Zl = Zl.t().contiguous().t()
                    E.unmtr_hb2st(F2, Zl)
                    lb.data[:n, :lb.nloc].copy_(Zl)
            Zc.storage.mark_local_modified(Zc.storage.origin_slot)
            # Q1 needs Z on F's row distribution (tile size = band)
            same = Z.storage.bc.mb == nb and Z.storage.bc.p == F.storage.bc.p
            Zg = Z if same else _new_general(F, n, n)
            if Z1 is not None or not same:
                redistribute(Z1 if Z1 is not None else Z, Zg)
            unmtr_he2hb_dist(F, Fac, Zg)
            if Zg is not Z:
                redistribute(Zg, Z)
        if sc != 1.0:
            w = w / sc
        if Lambda is not None:
            Lambda.copy_(w.to(Lambda.dtype).to(Lambda.device))
        return w


# bytes each path moved (tests: the host path carries O(n) words only)
BCAST_STATS = {"host_bytes": 0, "host_max": 0, "dev_bytes": 0}


def _bcast_host(comm, t, root):
    """Broadcast a small host tensor (staged through the GPU under RCCL)."""
    if comm.size == 1:
        return t
    x = t.clone()
    nbytes = x.numel() * x.element_size()
    BCAST_STATS["host_bytes"] += nbytes
    BCAST_STATS["host_max"] = max(BCAST_STATS["host_max"], nbytes)
    comm.bcast(x, root)
    return x


def _bcast_dev(comm, t, root, dev):
    """Broadcast a tensor that lives on ``dev`` (the GPU under RCCL: no host
    staging; the root's tensor is moved there once if it is not)."""
    if comm.size == 1:
        return t
    x = t.to(dev).contiguous()
    BCAST_STATS["dev_bytes"] += x.numel() * x.element_size()
    comm.bcast(x, root)
    return x
