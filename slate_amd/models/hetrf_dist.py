"""Distributed blocked Aasen (hetrf / hetrs on a p x q process grid): no
rank ever holds the dense matrix.

Reference: src/hetrf.cc:165-511 (the communication-avoiding Aasen: H = T
L^H per block column, the panel A(j1:, J) - L H, its LU with partial
pivoting via internal::getrf_panel, the symmetric interchange
permuteRowsCols, T(J+1, J) from the panel's U), src/hetrs.cc:94-105.

Data layout (MI355X design): the full Hermitian A (both triangles) and L
are block-cyclic on the grid with the tile size as the Aasen block nb; the
block tridiagonal T (Td, Tl: 2 N nb entries) is replicated, so H(0:J+1, J)
= T L(J, 0:J+1)^H is formed redundantly on every rank with three strided
batched MFMA GEMMs from the replicated block row L(J, 0:J+1) (one
all-reduce of nb x j1 per step).  Per step:

  * panel  : every rank multiplies its local rows of L(j1:, 0:j1) by the
             rows of H that match its local columns (one GEMM), the partial
             sums are reduced along the process row onto the panel's process
             column, which adds A(j1:, J) -- a stationary-L product, no L
             block ever moves;
  * LU     : the panel is all-gathered inside that process column and
             factored redundantly by the GPU partial-pivoting LU (identical
             pivots on every rank of the column); the new block column of L
             travels one row broadcast to its owners, T(J+1, J) and the
             pivots to everyone;
  * swaps  : the symmetric interchange P S P^T of the trailing A and the
             row interchange of L(j1:, 0:j1) are exact point-to-point moves
             of only the rows / columns that change process row / column
             (parallel/perm.py).

T is then factored redundantly by the band LU on every rank (N x 3nb).
hetrs: P b and P^T x by the same exact exchanges, the two triangular
solves by the distributed trsm, the band solve on a 1 x P column layout of
the right-hand sides (each rank solves its own columns; one redistribution
each way).
"""
from __future__ import annotations

import numpy as np
import torch

from .. import ops
from ..core.enums import Diag, Op, Side, Uplo
from ..core.exceptions import SlateError
from ..parallel.perm import exchange_lines, moves_from_ipiv, moves_from_perm
from ..utils.trace import trace_block
from ._util import conj_trans, grid_of, tiles_local_before


class DistIndefiniteFactors:
    def __init__(self, L, Tband, Tpiv, perm, n, N, nb, Td, Tl):
        self.L, self.Tband, self.Tpiv, self.perm = L, Tband, Tpiv, perm
        self.n, self.N, self.nb = n, N, nb
        self.Td, self.Tl = Td, Tl
        self.distributed = True


def _blk(S, I, nb):
    return S[:, I * nb:(I + 1) * nb]


def _gcols(nloc, nb, q, pc):
    """Global indices of the nloc local columns of process column pc."""
    lc = np.arange(nloc, dtype=np.int64)
    return ((lc // nb) * q + pc) * nb + lc % nb


def _full_padded(A, N, nb, slot):
    """The full Hermitian A (both triangles) as an N x N general
    block-cyclic matrix on A's grid, identity on the padding."""
    from .blas3 import _fresh, _full_from_stored
    from ..parallel.redist import redistribute_pieces
    n = A.n()
    F = _full_from_stored(A, slot, herm=A._kind != "symmetric")
    if N == n:
        return F
    G = _fresh(F, N, N, slot)
    redistribute_pieces(F, G.slice(0, n - 1, 0, n - 1))
    from .aux import set_diag
    set_diag(G.slice(n, N - 1, n, N - 1), 1.0)
    return G


def hetrf_dist(A, opts=None):
    """Returns (info, DistIndefiniteFactors); A is left untouched except for
    the factors attached by hetrf()."""
    from .blas3 import _fresh
    from ._util import target_slot
    s = A.storage
    bc = s.bc
    if bc is None or bc.mb != bc.nb:
        raise SlateError("hetrf (distributed): square-tile block-cyclic A required")
    slot = target_slot(A, opts)
    nb = bc.nb
    n = A.n()
    N = -(-max(n, 1) // nb) * nb
    NT = N // nb
    with trace_block("hetrf_dist"):
        F = _full_padded(A, N, nb, slot)
        L = _fresh(F, N, N, slot)
        fb, lb = F.local_block(slot), L.local_block(slot)
        fl, ll = fb.data, lb.data
        dev, dt = fl.device, s.dtype
        sF = F.storage.bc
        p, q, pr, pc = sF.p, sF.q, sF.pr, sF.pc
        mloc, nloc = fb.mloc, fb.nloc
        grid = grid_of(F)
        comm = F.storage.comm
        ct = conj_trans(dt)
        gcol = torch.from_numpy(_gcols(nloc, nb, q, pc)).to(dev)
        # L(0:nb, 0:nb) = I on its owner
        if pr == 0 and pc == 0:
            ops.geset(0.0, 1.0, ll[:nb, :nb])
        Td = ops.colmajor_zeros(nb, NT * nb, dt, dev)
        Tl = ops.colmajor_zeros(nb, (NT + 1) * nb, dt, dev)
        Xs = ops.colmajor_zeros(N, nb, dt, dev)
        Hs = ops.colmajor_zeros(N, nb, dt, dev)
        S = ops.colmajor_empty(nb, nb, dt, dev)
        tmp = ops.colmajor_empty(nb, nb, dt, dev)
        ipiv = np.arange(N, dtype=np.int64)
        for J in range(NT):
            j0, j1 = J * nb, (J + 1) * nb
            rJ, cJ = J % p, J % q
            lrJ = tiles_local_before(J, p, pr) * nb
            lr1 = min(tiles_local_before(J + 1, p, pr) * nb, mloc)
            lc1 = min(tiles_local_before(J + 1, q, pc) * nb, nloc)
            # ---- block row J of L (cols < j1) and A(J, J), replicated
            with trace_block("hetrf::row"):
                R = torch.zeros(nb, j1 + nb, dtype=dt, device=dev)
                if pr == rJ:
                    if lc1:
                        R[:, :j1].index_copy_(1, gcol[:lc1], ll[lrJ:lrJ + nb, :lc1])
                    if pc == cJ:
                        lcJ = tiles_local_before(J, q, pc) * nb
                        R[:, j1:].copy_(fl[lrJ:lrJ + nb, lcJ:lcJ + nb])
                if comm.size > 1:
                    comm.allreduce(R)
                Lrow = ops.colmajor_empty(nb, j1, dt, dev)
                Lrow.copy_(R[:, :j1])
                Ajj = R[:, j1:]
                ops.gecopy(Lrow, Xs[0:j1], trans='C')
            # ---- H(0:J, J) = T X (replicated, batched GEMMs as the 1-rank form)
            with trace_block("hetrf::H"):
                if J > 0:
                    ops.gemm(1.0, _blk(Td, 0, nb), Xs[0:nb], 0.0, Hs[0:nb], batch=J, strides=(nb * nb, nb, nb))
                    if J > 1:
                        ops.gemm(1.0, _blk(Tl, 1, nb), Xs[0:nb], 1.0, Hs[nb:2 * nb], batch=J - 1,
                                 strides=(nb * nb, nb, nb))
                    ops.gemm(1.0, _blk(Tl, 1, nb), Xs[nb:2 * nb], 1.0, Hs[0:nb], transA=ct, batch=J,
                             strides=(nb * nb, nb, nb))
                S.copy_(Ajj)
                Ljj = Lrow[:, j0:j1]
                if J > 0:
                    ops.gemm(-1.0, Lrow[:, 0:j0], Hs[0:j0], 1.0, S)
                    ops.gemm(1.0, _blk(Tl, J, nb), Xs[j0 - nb:j0], 0.0, tmp)
                    ops.gemm(-1.0, Ljj, tmp, 1.0, S)
                    ops.trsm('L', 'L', 'N', 'U', 1.0, Ljj, S)
                    ops.trsm('R', 'L', ct, 'U', 1.0, Ljj, S)
                ops.gecopy(S, tmp, trans='C')
                ops.geadd(0.5, tmp, 0.5, S)
                _blk(Td, J, nb).copy_(S)
                ops.gemm(1.0, S, Xs[j0:j1], 0.0, Hs[j0:j1])
                if J > 0:
                    ops.gemm(1.0, _blk(Tl, J, nb), Xs[j0 - nb:j0], 1.0, Hs[j0:j1])
            if J == NT - 1:
                break
            # ---- panel W = A(j1:, J) - L(j1:, 0:j1) H(0:j1, J) on process column cJ
            with trace_block("hetrf::panel"):
                nmine = mloc - lr1
                W = ops.colmajor_zeros(nmine, nb, dt, dev)
                if nmine and lc1:
                    Hsel = ops.colmajor_empty(lc1, nb, dt, dev)
                    ops.row_gather(Hs, Hsel, gcol[:lc1])
                    ops.gemm(-1.0, ll[lr1:mloc, :lc1], Hsel, 0.0, W)
                if q > 1 and nmine:
                    grid.row_comm.reduce(W, cJ)
                piv_t = torch.zeros(nb + 1, dtype=torch.int64, device=dev)     # pivots + info
                T1 = ops.colmajor_zeros(nb, nb, dt, dev)
                Lpan = None
                if pc == cJ:
                    lcJ = tiles_local_before(J, q, pc) * nb
                    if nmine:
                        ops.geadd(1.0, fl[lr1:mloc, lcJ:lcJ + nb], 1.0, W)
                    Pn, rows_of = _gather_panel(W, grid, J + 1, nb, p, pr, N, mloc, dt, dev)
                    piv = piv_t[:nb]
                    ops.getrf(Pn, piv, piv_t[nb:nb + 1])
                    Lfull = ops.colmajor_zeros(N - j1, nb, dt, dev)
                    ops.v_explicit(Pn, Lfull)
                    ops.gecopy(Pn[0:nb], T1, uplo='U')                   # T1 zero below
                    ops.trsm('R', 'L', ct, 'U', 1.0, Ljj, T1)
                    # this process row's rows of the new L block column
                    Lpan = ops.colmajor_empty(nmine, nb, dt, dev)
                    if nmine:
                        ops.row_gather(Lfull, Lpan, rows_of)
                # pivots + T1 to everyone (the panel's process column computed
                # them redundantly), the L block column along each row
                if q > 1:
                    grid.row_comm.bcast(piv_t, cJ)
                    grid.row_comm.bcast(T1, cJ)
                _blk(Tl, J + 1, nb).copy_(T1)
                if Lpan is None:
                    Lpan = ops.colmajor_empty(nmine, nb, dt, dev)
                if q > 1 and nmine:
                    grid.row_comm.bcast(Lpan, cJ)
                cJ1 = (J + 1) % q
                if pc == cJ1 and nmine:
                    lcJ1 = tiles_local_before(J + 1, q, pc) * nb
                    ll[lr1:mloc, lcJ1:lcJ1 + nb].copy_(Lpan)
                ph = piv_t.cpu().numpy()                      # host: the exchange plan
            # ---- symmetric interchange of the trailing A, rows of L(j1:, 0:j1)
            with trace_block("hetrf::swap"):
                mv = moves_from_ipiv(ph[:nb] + j1, j1)
                ipiv[j1:j1 + nb] = ph[:nb] + j1
                if mv:
                    exchange_lines(grid.col_comm, ll[:mloc, :lc1], mv, nb, p, pr, 0)
                    exchange_lines(grid.col_comm, fl[:mloc, lc1:nloc], mv, nb, p, pr, 0)
                    exchange_lines(grid.row_comm, fl[lr1:mloc, :nloc], mv, nb, q, pc, 1)
        L.storage.mark_local_modified(L.storage.origin_slot)
        perm = _perm_of(ipiv, N)
        from .hetrf import _band_T
        Tb = _band_T(Td, Tl, N, nb, dt, dev)
        from ..core.matrix import Pivots
        from .band import gbtrf
        Tpiv = Pivots()
        info_t = gbtrf(Tb, Tpiv)
        return int(info_t), DistIndefiniteFactors(L, Tb, Tpiv, perm, n, N, nb, Td, Tl)


def _gather_panel(W, grid, t0, nb, p, pr, N, mloc, dt, dev):
    """All-gather the panel rows (global tile rows >= t0) inside the process
    column: returns (the panel, global order, N - t0 nb rows; the panel rows
    of this rank's local rows)."""
    from ..core.storage import numroc
    from ._panels import rows_global
    r0 = t0 * nb
    cnt = [max(0, numroc(N, nb, r, p) - min(tiles_local_before(t0, p, r) * nb, numroc(N, nb, r, p)))
           for r in range(p)]
    mx = max(max(cnt), 1)
    pad = ops.colmajor_zeros(mx, nb, dt, dev)
    if W.shape[0]:
        pad[:W.shape[0]].copy_(W)
    allp = grid.col_comm.allgather(pad.t().contiguous()) if p > 1 else pad.t().unsqueeze(0)
    Pn = ops.colmajor_empty(N - r0, nb, dt, dev)
    for r in range(p):
        if cnt[r]:
            lr0 = tiles_local_before(t0, p, r) * nb
            ops.row_scatter(allp[r].t()[:cnt[r]], Pn, rows_global(lr0, lr0 + cnt[r], nb, p, r, r0, dev))
    lr0 = min(tiles_local_before(t0, p, pr) * nb, mloc)
    mine = rows_global(lr0, mloc, nb, p, pr, r0, dev)
    return Pn, mine


def _perm_of(ipiv, N):
    perm = np.arange(N, dtype=np.int64)
    for i, j in enumerate(ipiv.tolist()):
        if j != i:
            perm[i], perm[j] = perm[j], perm[i]
    return perm


def hetrs_dist(Fac, B, opts=None):
    """x = P^T L^{-H} T^{-1} L^{-1} P b on the grid (B overwritten)."""
    from .blas3 import _fresh, trsm
    from ..core.matrix import Matrix, TriangularMatrix
    from ..parallel.redist import redistribute_pieces
    from ._util import target_slot
    from .band import gbtrs
    from ..parallel import comm as _comm
    L = Fac.L
    n, N, nb = Fac.n, Fac.N, Fac.nb
    nr = B.n()
    slot = target_slot(L, opts)
    with trace_block("hetrs_dist"):
        Y = _fresh(L, N, nr, slot)
        redistribute_pieces(B, Y.slice(0, n - 1, 0, nr - 1))
        lbY = Y.local_block(slot)
        bcY = Y.storage.bc
        grid = grid_of(Y)
        mv = moves_from_perm(Fac.perm)
        if mv and lbY.nloc:
            exchange_lines(grid.col_comm, lbY.data[:lbY.mloc, :lbY.nloc], mv, nb, bcY.p, bcY.pr, 0)
        Lt = TriangularMatrix(Uplo.Lower, L, diag=Diag.Unit)
        trsm(Side.Left, 1.0, Lt, Y, opts)
        # band solve: each rank solves whole columns of a 1 x P layout
        P = Y.storage.comm.size
        Yc = Matrix(N, nr, nb=nb, p=1, q=P, comm=Y.storage.comm, dtype=Y.storage.dtype,
                    device=lbY.data.device)
        Yc.insertLocalTiles(device=lbY.data.device if lbY.data.is_cuda else -1)
        redistribute_pieces(Y, Yc)
        lc = Yc.local_block(slot)
        if lc.nloc:
            Z = Matrix(N, lc.nloc, nb=nb, p=1, q=1, comm=_comm.self_comm(), dtype=Y.storage.dtype,
                       device=lc.data.device)
            Z.insertLocalTiles(device=lc.data.device if lc.data.is_cuda else -1)
            Z.local_block().data[:N, :lc.nloc].copy_(lc.data[:N, :lc.nloc])
            gbtrs(Fac.Tband, Fac.Tpiv, Z)
            lc.data[:N, :lc.nloc].copy_(Z.local_block().data[:N, :lc.nloc])
        Yc.storage.mark_local_modified(Yc.storage.origin_slot)
        redistribute_pieces(Yc, Y)
        trsm(Side.Left, 1.0, Lt.conj_transpose(), Y, opts)
        inv = np.empty_like(Fac.perm)
        inv[Fac.perm] = np.arange(N)
        mv = moves_from_perm(inv)
        lbY = Y.local_block(slot)
        if mv and lbY.nloc:
            exchange_lines(grid.col_comm, lbY.data[:lbY.mloc, :lbY.nloc], mv, nb, bcY.p, bcY.pr, 0)
        Y.storage.mark_local_modified(Y.storage.origin_slot)
        redistribute_pieces(Y.slice(0, n - 1, 0, nr - 1), B)
    return 0
