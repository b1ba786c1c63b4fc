"""Symmetric/Hermitian indefinite solvers: hetrf / hetrs / hesv (and the
sy* aliases) -- P A P^H = L T L^H with T Hermitian BLOCK tridiagonal
(bandwidth nb), factored afterwards by the band LU.

Reference: `src/hetrf.cc` (communication-avoiding blocked Aasen, host
only: "GPU version not yet implemented", `src/hetrf.cc:23`; band T
factored by gbtrf, `:511`), `src/hetrs.cc:94-105` (trsm + gbtrs + trsm),
`src/hesv.cc`.

MI355X design: the blocked left-looking Aasen algorithm (Rozloznik,
Shklarski, Toledo; Ballard et al.), every step a handful of device
launches -- no per-column work on the host:

  step J (block column j0:j1, H = T L^H, L(:, 0) = [I; 0]):
    H(0:J, J)  = the block-tridiagonal T times L(J, 0:J+1)^H: three
                 strided-BATCHED MFMA GEMMs (one launch per diagonal);
    T(J, J)    = L(J,J)^{-1} (A(J,J) - L(J,0:J) H(0:J,J)
                 - L(J,J) T(J,J-1) L(J,J-1)^H) L(J,J)^{-H}  (GEMM + 2 trsm);
    panel      = A(j1:, J) - L(j1:, 0:j1) H(0:j1, J)          (one GEMM);
    LU with partial pivoting of the panel (the GPU recursive/persistent
    getrf): L(j1:, J+1) and T(J+1, J) = U L(J,J)^{-H};
    symmetric interchange of the trailing A: row laswp, conjugate
    transpose copy, row laswp (P S P^T = P (P S)^H for Hermitian S).

The order is padded to a multiple of nb with an identity block (never
selected as pivot).  T is stored as compact band storage and factored by
gbtrf (models/band.py); hetrs is trsm + gbtrs + trsm.  On a process grid
the distributed form in models/hetrf_dist.py runs instead (no rank holds
the dense matrix).
"""
from __future__ import annotations

import torch

from .. import ops
from ..core.enums import Uplo
from ..core.matrix import Pivots
from ..utils.trace import trace_block
from ._util import conj_trans
from .aux import allgather_dense, from_dense


class IndefiniteFactors:
    """Device factors of hetrf: L (N x N unit lower, first block column
    [I; 0]), the band LU of T (BandMatrix + pivots), the permutation perm
    (row i of P A is row perm[i] of A) and the padded order N >= n."""

    def __init__(self, L, Tband, Tpiv, perm, n, N, nb, Td, Tl):
        self.L, self.Tband, self.Tpiv, self.perm = L, Tband, Tpiv, perm
        self.n, self.N, self.nb = n, N, nb
        self.Td, self.Tl = Td, Tl


def _full(A):
    from .eig import _dense_hermitian
    return _dense_hermitian(A)


def _blk(S, I, nb):
    """Block I of a (nb x NT nb) column-major stack."""
    return S[:, I * nb:(I + 1) * nb]


def aasen(Af: torch.Tensor, nb: int):
    """Blocked Aasen on the dense Hermitian Af (N x N, both triangles,
    N % nb == 0; overwritten).  Returns (L, Td, Tl, ipiv) with ipiv the
    global 0-based interchange sequence (LAPACK style)."""
    N = Af.shape[0]
    NT = N // nb
    dt, dev = Af.dtype, Af.device
    ct = conj_trans(dt)
    L = ops.colmajor_zeros(N, N, dt, dev)
    ops.geset(0.0, 1.0, L[:nb, :nb])
    Td = ops.colmajor_zeros(nb, NT * nb, dt, dev)
    Tl = ops.colmajor_zeros(nb, (NT + 1) * nb, dt, dev)       # Tl[I] = T(I, I-1); Tl[0] = 0
    Xs = ops.colmajor_zeros(N, nb, dt, dev)                    # L(J, 0:J+1)^H stacked
    Hs = ops.colmajor_zeros(N, nb, dt, dev)                    # H(0:J+1, J) stacked
    S = ops.colmajor_empty(nb, nb, dt, dev)
    tmp = ops.colmajor_empty(nb, nb, dt, dev)
    Wt = ops.colmajor_empty(N, N, dt, dev)                     # transpose workspace
    ipiv = torch.arange(N, dtype=torch.int64).to(dev)         # block 0: no interchanges (host iota, one copy)
    info = torch.zeros(max(NT, 1), dtype=torch.int64, device=dev)
    for J in range(NT):
        j0, j1 = J * nb, (J + 1) * nb
        with trace_block("hetrf::H"):
            ops.gecopy(L[j0:j1, 0:j1], Xs[0:j1], trans='C')
            if J > 0:
                # H(I, J) = Td[I] X[I] + Tl[I] X[I-1] + Tl[I+1]^H X[I+1], I < J
                ops.gemm(1.0, _blk(Td, 0, nb), Xs[0:nb], 0.0, Hs[0:nb], batch=J,
                         strides=(nb * nb, nb, nb))
                if J > 1:
                    ops.gemm(1.0, _blk(Tl, 1, nb), Xs[0:nb], 1.0, Hs[nb:2 * nb], batch=J - 1,
                             strides=(nb * nb, nb, nb))
                ops.gemm(1.0, _blk(Tl, 1, nb), Xs[nb:2 * nb], 1.0, Hs[0:nb], transA=ct, batch=J,
                         strides=(nb * nb, nb, nb))
        with trace_block("hetrf::T"):
            S.copy_(Af[j0:j1, j0:j1])
            Ljj = L[j0:j1, j0:j1]
            if J > 0:
                ops.gemm(-1.0, L[j0:j1, 0:j0], Hs[0:j0], 1.0, S)
                ops.gemm(1.0, _blk(Tl, J, nb), Xs[j0 - nb:j0], 0.0, tmp)          # Tl[J] L(J,J-1)^H
                ops.gemm(-1.0, Ljj, tmp, 1.0, S)
                ops.trsm('L', 'L', 'N', 'U', 1.0, Ljj, S)
                ops.trsm('R', 'L', ct, 'U', 1.0, Ljj, S)
            # Hermitian part (rounding): Td[J] = (S + S^H) / 2
            ops.gecopy(S, tmp, trans='C')
            ops.geadd(0.5, tmp, 0.5, S)
            _blk(Td, J, nb).copy_(S)
            # H(J, J) = Tl[J] L(J,J-1)^H + Td[J] L(J,J)^H
            ops.gemm(1.0, S, Xs[j0:j1], 0.0, Hs[j0:j1])
            if J > 0:
                ops.gemm(1.0, _blk(Tl, J, nb), Xs[j0 - nb:j0], 1.0, Hs[j0:j1])
        if J == NT - 1:
            break
        with trace_block("hetrf::panel"):
            Wp = Af[j1:N, j0:j1]
            ops.gemm(-1.0, L[j1:N, 0:j1], Hs[0:j1], 1.0, Wp)
            piv = ipiv[j1:j1 + nb]
            ops.getrf(Wp, piv, info[J:J + 1])
            ops.v_explicit(Wp, L[j1:N, j1:j1 + nb])
            T1 = _blk(Tl, J + 1, nb)
            ops.geset(0.0, 0.0, T1)
            ops.gecopy(Wp[0:nb], T1, uplo='U')
            ops.trsm('R', 'L', ct, 'U', 1.0, Ljj, T1)
        with trace_block("hetrf::swap"):
            ops.laswp(L[j1:N, 0:j1], piv, 0, nb)
            Str = Af[j1:N, j1:N]
            ops.laswp(Str, piv, 0, nb)
            Wv = Wt[0:N - j1, 0:N - j1]
            ops.gecopy(Str, Wv, trans='C')
            ops.laswp(Wv, piv, 0, nb)
            Str.copy_(Wv)
    # panel-relative -> global interchange indices: one host pass (the caller
    # reads ipiv on the host anyway)
    ipiv = ipiv.cpu()
    for j1 in range(nb, N, nb):
        ipiv[j1:j1 + nb] += j1
    return L, Td, Tl, ipiv


def _perm_of(ipiv_host, N):
    perm = list(range(N))
    for i, j in enumerate(ipiv_host):
        if j != i:
            perm[i], perm[j] = perm[j], perm[i]
    return perm


def _band_T(Td, Tl, N, nb, dt, dev):
    """The block-tridiagonal T as a compact band matrix (kl = ku = nb) on
    this rank alone."""
    from ..core.matrix import BandMatrix
    from ..parallel import comm as _comm
    from ..core.storage import DEV, HOST
    Tb = BandMatrix(N, N, nb, nb, nb=nb, comm=_comm.self_comm(), dtype=dt, device=dev)
    Tb.insertLocalTiles(device=dev.index if dev.type == "cuda" else -1)
    s = Tb.storage
    slot = s.band_slot()
    NT = N // nb
    for J in range(NT):
        s.tiles[(J, J, slot)].copy_(_blk(Td, J, nb))
        if J + 1 < NT:
            lo = _blk(Tl, J + 1, nb)                                  # T(J+1, J), upper triangular
            s.tiles[(J + 1, J, slot)].copy_(lo)
            up = s.tiles[(J, J + 1, slot)]
            ops.gecopy(lo, up, trans='C')                              # T(J, J+1) = T(J+1, J)^H
    s.mark_local_modified(slot)
    return Tb


def hetrf(A, pivots: Pivots = None, T=None, pivots2=None, H=None, opts=None):
    """Factor the Hermitian indefinite A: P A P^H = L T L^H (blocked Aasen,
    see module docstring).  L (unit lower, first block column [I; 0])
    overwrites the strictly lower part of A from block column 1 on (shifted
    one block left, as SLATE); the permutation goes to ``pivots``, the
    block-tridiagonal T to the band matrix ``T`` if given.  Returns info."""
    from .band import gbtrf
    s = A.storage
    if s.comm.size > 1 and s.bc is not None and s.bc.mb == s.bc.nb:
        # on a grid: the distributed Aasen (models/hetrf_dist.py), no gather
        from .hetrf_dist import hetrf_dist
        info, F = hetrf_dist(A, opts)
        A._hetrf = F
        if pivots is not None:
            pivots.set(torch.as_tensor(F.perm[:F.n].copy(), dtype=torch.int64), 1)
        return info
    with trace_block("hetrf"):
        s = A.storage
        n = A.n()
        nb = max(8, min(s.tileNb(0) if s.nt else 64, 256))
        N = -(-max(n, 1) // nb) * nb
        dev = s.device if s.device.type == "cuda" else torch.device("cpu")
        dt = s.dtype
        Af = ops.colmajor_zeros(N, N, dt, dev)
        Af[:n, :n].copy_(_full(A).to(dev))
        if N > n:
            ops.geset(0.0, 1.0, Af[n:, n:])
        L, Td, Tl, ipiv = aasen(Af, nb)
        ip = ipiv.cpu().tolist()
        perm = torch.as_tensor(_perm_of(ip, N), dtype=torch.int64, device=dev)
        Tb = _band_T(Td, Tl, N, nb, dt, dev)
        if T is not None:
            from .band import _is_band
            D = torch.zeros(N, N, dtype=dt, device=dev)
            for J in range(N // nb):
                D[J * nb:(J + 1) * nb, J * nb:(J + 1) * nb] = _blk(Td, J, nb)
                if J + 1 < N // nb:
                    D[(J + 1) * nb:(J + 2) * nb, J * nb:(J + 1) * nb] = _blk(Tl, J + 1, nb)
                    D[J * nb:(J + 1) * nb, (J + 1) * nb:(J + 2) * nb] = _blk(Tl, J + 1, nb).mH
            if _is_band(T) or T.m() == n:
                from_dense(T, D[:n, :n])
        Tpiv = Pivots()
        info = gbtrf(Tb, Tpiv)
        A._hetrf = IndefiniteFactors(L, Tb, Tpiv, perm, n, N, nb, Td, Tl)
        # L below the first block column, shifted one block left (SLATE layout)
        # (triangle copies and clears are tile-kernel launches: gecopy / geset)
        out = ops.colmajor_zeros(n, n, dt, dev)
        if N > nb:
            ov = out[nb:n, 0:n - nb]
            ops.gecopy(L[nb:n, nb:n], ov, uplo='L')
            ops.geset(0.0, 0.0, ov, uplo='U')           # strictly lower part of L only
        for J in range(N // nb):
            r0, r1 = J * nb, min(n, (J + 1) * nb)
            if r0 < n:
                ob = out[r0:r1, r0:r1]
                ops.geset(0.0, 0.0, ob)
                ops.gecopy(_blk(Td, J, nb)[:r1 - r0, :r1 - r0], ob, uplo='L')
        up = A.uploPhysical()
        from_dense(A, out if up != Uplo.Upper else out.mH)
        if pivots is not None:
            pivots.set(perm[:n].clone(), 1)
        return int(info)


def hetrs(A, pivots=None, T=None, pivots2=None, B=None, opts=None):
    """Solve A X = B with the factors of hetrf (B overwritten):
    x = P^T L^{-H} T^{-1} L^{-1} P b."""
    from .band import gbtrs
    if getattr(A._hetrf, "distributed", False):
        from .hetrf_dist import hetrs_dist
        return hetrs_dist(A._hetrf, B, opts)
    with trace_block("hetrs"):
        F = A._hetrf
        dev = F.L.device
        n, N = F.n, F.N
        Bd = allgather_dense(B).to(dev)
        nr = Bd.shape[1]
        Y = ops.colmajor_zeros(N, nr, Bd.dtype, dev)
        Y[:n].copy_(Bd)
        Yp = ops.colmajor_empty(N, nr, Bd.dtype, dev)
        ops.row_gather(Y, Yp, F.perm)                     # P b
        ops.trsm('L', 'L', 'N', 'U', 1.0, F.L, Yp)
        from ..core.matrix import Matrix
        from ..parallel import comm as _comm
        Z = Matrix(N, nr, nb=F.nb, p=1, q=1, comm=_comm.self_comm(), dtype=Bd.dtype, device=dev)
        Z.insertLocalTiles(device=dev.index if dev.type == "cuda" else -1)
        from_dense(Z, Yp)
        gbtrs(F.Tband, F.Tpiv, Z)
        Zd = Z.local_block().data[:N, :nr]
        Zc = ops.colmajor_empty(N, nr, Bd.dtype, dev)
        Zc.copy_(Zd)
        ops.trsm('L', 'L', conj_trans(Bd.dtype), 'U', 1.0, F.L, Zc)
        X = ops.colmajor_empty(N, nr, Bd.dtype, dev)
        ops.row_scatter(Zc, X, F.perm)                    # P^T
        from_dense(B, X[:n])
        return 0


def hesv(A, pivots=None, T=None, pivots2=None, H=None, B=None, opts=None) -> int:
    info = hetrf(A, pivots, T, pivots2, H, opts)
    if info == 0:
        hetrs(A, pivots, T, pivots2, B, opts)
    return info


sytrf = hetrf
sytrs = hetrs
sysv = hesv
