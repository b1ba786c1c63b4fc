"""Band drivers: gbtrf / gbtrs / gbsv (band LU with partial pivoting),
pbtrf / pbtrs / pbsv (band Cholesky), gbmm, hbmm, tbsm.

Reference: `src/gbtrf.cc:20-348` (panel + band-limited trailing update,
upper bandwidth grows to kl+ku), `src/gbtrs.cc`, `src/gbsv.cc`,
`src/pbtrf.cc`, `src/pbtrs.cc`, `src/pbsv.cc`, `src/gbmm.cc`, `src/hbmm.cc`,
`src/tbsm.cc`, `src/tbsmPivots.cc`.

MI355X design: band matrices use the same block-cyclic local buffer as
general ones (SLATE also stores whole tiles).  On one rank the
factorizations run a band-limited step loop directly on the device buffer
(the GPU LU panel over the kb+kl rows that can be non-zero, trailing TRSM +
MFMA GEMM only inside the (kl+ku)-wide window), so the cost is
O(n kl (kl+ku)) not O(n^3).  On a grid, entries outside the band are
zeroed and the dense distributed drivers run (pivot rows can never leave
the band because all rows below it are zero, so the result is the band
factorization).  Solves and products go through the dense drivers on the
zero-masked operands.
"""
from __future__ import annotations

import torch

from .. import ops
from ..core.enums import Diag, Side, Uplo
from ..core.matrix import Pivots, TriangularMatrix
from ..utils.trace import trace_block


def _bands(A):
    kl = A.lowerBandwidth() if hasattr(A, "lowerBandwidth") else A.m()
    ku = A.upperBandwidth() if hasattr(A, "upperBandwidth") else A.n()
    return kl, ku


def band_mask(A, kl=None, ku=None):
    """Zero every local entry outside -ku <= i - j <= kl (global indices)."""
    s = A.storage
    if kl is None:
        kl, ku = _bands(A)
    lb = A.local_block()
    if lb.mloc == 0 or lb.nloc == 0:
        return A
    dev = lb.data.device
    gr = torch.tensor([lb.global_row(i) for i in range(lb.mloc)], device=dev)
    gc = torch.tensor([lb.global_col(j) for j in range(lb.nloc)], device=dev)
    d = gr[:, None] - gc[None, :]
    outside = (d > kl) | (d < -ku)
    lb.data.masked_fill_(outside, 0)
    s.mark_local_modified(s.origin_slot)
    return A


def _single(A):
    s = A.storage
    return s.comm.size == 1 or (s.bc is not None and s.bc.p * s.bc.q == 1)


# ------------------------------------------------------------------ LU
def gbtrf(A, pivots: Pivots, opts=None) -> int:
    """Band LU with partial pivoting; pivots are global row indices."""
    from .lu import getrf
    with trace_block("gbtrf"):
        kl, ku = _bands(A)
        band_mask(A, kl, ku)
        if not _single(A):
            info = getrf(A, pivots, opts)
            return info
        s = A.storage
        from ._util import target_slot
        slot = target_slot(A, opts)
        buf = s.prepare_local(slot)
        m, n = s.m, s.n
        nb = s.bc.nb
        kt = (min(m, n) + nb - 1) // nb
        dev = buf.device
        ipiv = torch.zeros(max(min(m, n), 1), dtype=torch.int64, device=dev)
        infos = torch.zeros(max(kt, 1), dtype=torch.int64, device=dev)
        for k in range(kt):
            r0 = k * nb
            kb = min(nb, n - r0, m - r0)
            rend = min(m, r0 + kb + kl)
            cend = min(n, r0 + kb + kl + ku)
            piv = ipiv[r0:r0 + kb]
            ops.getrf(buf[r0:rend, r0:r0 + kb], piv, infos[k:k + 1])
            if r0 > 0:
                ops.laswp(buf[:m, 0:r0], ipiv, r0, r0 + kb, ioff=-r0)
            if cend > r0 + kb:
                C = buf[:m, r0 + kb:cend]
                ops.laswp(C, ipiv, r0, r0 + kb, ioff=-r0)
                ops.trsm('L', 'L', 'N', 'U', 1.0, buf[r0:r0 + kb, r0:r0 + kb], buf[r0:r0 + kb, r0 + kb:cend])
                if rend > r0 + kb:
                    ops.gemm(-1.0, buf[r0 + kb:rend, r0:r0 + kb], buf[r0:r0 + kb, r0 + kb:cend], 1.0,
                             buf[r0 + kb:rend, r0 + kb:cend])
        s.mark_local_modified(slot)
        glob = ipiv.clone()
        for k in range(kt):
            r0 = k * nb
            kb = min(nb, n - r0, m - r0)
            glob[r0:r0 + kb] += r0
        pivots.set(glob[:min(m, n)], nb)
        iv = infos[:kt].cpu().tolist()
        for k, v in enumerate(iv):
            if v > 0:
                return k * nb + v
        return 0


def gbtrs(A, pivots, B, opts=None):
    from .lu import getrs
    with trace_block("gbtrs"):
        return getrs(A, pivots, B, opts)


def gbsv(A, pivots, B, opts=None) -> int:
    info = gbtrf(A, pivots, opts)
    if info == 0:
        gbtrs(A, pivots, B, opts)
    return info


# ------------------------------------------------------------------ Cholesky
def pbtrf(A, opts=None) -> int:
    """Band Cholesky of a Hermitian band matrix (kd = bandwidth)."""
    from .chol import potrf
    with trace_block("pbtrf"):
        kd = getattr(A, "_kd", max(_bands(A)))
        if A.uploPhysical() == Uplo.Lower:
            band_mask(A, kd, 0)
        else:
            band_mask(A, 0, kd)
        if not _single(A) or A.uploPhysical() != Uplo.Lower:
            return potrf(A, opts)
        s = A.storage
        from ._util import target_slot
        slot = target_slot(A, opts)
        buf = s.prepare_local(slot)
        n = s.n
        nb = s.bc.nb
        dev = buf.device
        kt = (n + nb - 1) // nb
        infos = torch.zeros(max(kt, 1), dtype=torch.int64, device=dev)
        ct = 'C' if s.dtype.is_complex else 'T'
        for k in range(kt):
            r0 = k * nb
            kb = min(nb, n - r0)
            rend = min(n, r0 + kb + kd)
            ops.potrf('L', buf[r0:r0 + kb, r0:r0 + kb], infos[k:k + 1])
            if rend > r0 + kb:
                P = buf[r0 + kb:rend, r0:r0 + kb]
                ops.trsm('R', 'L', ct, 'N', 1.0, buf[r0:r0 + kb, r0:r0 + kb], P)
                ops.gemm(-1.0, P, P, 1.0, buf[r0 + kb:rend, r0 + kb:rend], 'N', ct,
                         mask=(1, 1 << 40, 1, 0, 1, 0, 0, 0, 0))
        s.mark_local_modified(slot)
        iv = infos[:kt].cpu().tolist()
        for k, v in enumerate(iv):
            if v > 0:
                return k * nb + v
        return 0


def pbtrs(A, B, opts=None):
    from .chol import potrs
    with trace_block("pbtrs"):
        return potrs(A, B, opts)


def pbsv(A, B, opts=None) -> int:
    info = pbtrf(A, opts)
    if info == 0:
        pbtrs(A, B, opts)
    return info


# ------------------------------------------------------------------ BLAS-3
def gbmm(alpha, A, B, beta, C, opts=None):
    """C = alpha A B + beta C with A a band matrix."""
    from .blas3 import gemm
    with trace_block("gbmm"):
        band_mask(A)
        return gemm(alpha, A, B, beta, C, opts)


def hbmm(side, alpha, A, B, beta, C, opts=None):
    """C = alpha A B + beta C (Left) or alpha B A + beta C with A Hermitian band."""
    from .blas3 import hemm
    with trace_block("hbmm"):
        kd = getattr(A, "_kd", max(_bands(A)))
        band_mask(A, kd, 0) if A.uploPhysical() == Uplo.Lower else band_mask(A, 0, kd)
        return hemm(side, alpha, A, B, beta, C, opts)


def tbsm(side, alpha, A, B, pivots=None, opts=None):
    """Triangular band solve op(A) X = alpha B (optionally with the gbtrf
    row pivots applied to B first, tbsmPivots)."""
    from .blas3 import trsm
    from .lu import permute_rows
    with trace_block("tbsm"):
        kd = getattr(A, "_kd", max(_bands(A)))
        if pivots is not None:
            permute_rows(B, pivots, forward=True)
        band_mask(A, kd, 0) if A.uploPhysical() == Uplo.Lower else band_mask(A, 0, kd)
        return trsm(side, alpha, A, B, opts)
