"""Triangular inverse and product: trtri, trtrm (used by potri / getri).

Reference: `src/trtri.cc`, `src/trtrm.cc`, `internal_trtri.cc`,
`internal_trtrm.cc`, `src/potri.cc`.

MI355X design: on one GPU (or one rank) the inverse is the gfx950 tri_inv
kernel chain (block-diagonal 64x64 inverses + doubling MFMA GEMMs) and
trtrm is one trmm; on a grid both are expressed through the distributed
trsm/trmm drivers (T^{-1} = trsm(T, I)), so no separate communication
pattern is needed.
"""
from __future__ import annotations

import torch

from .. import ops
from ..core.enums import Diag, Side, Uplo
from ..core.exceptions import SlateError
from ..core.matrix import TriangularMatrix
from ..utils.trace import trace_block


def _single(A):
    s = A.storage
    return s.comm.size == 1 or (s.bc is not None and s.bc.p * s.bc.q == 1)


def trtri(A, opts=None) -> int:
    """In-place inverse of a triangular matrix; returns info (first zero
    diagonal, 1-based)."""
    with trace_block("trtri"):
        s = A.storage
        uplo = A.uploPhysical()
        diag = A.diag() if hasattr(A, "diag") else Diag.NonUnit
        dch = 'U' if diag == Diag.Unit else 'N'
        uch = 'L' if uplo == Uplo.Lower else 'U'
        n = A.n()
        if _single(A):
            lb = A.local_block()
            F = lb.data[:n, :n]
            info = ops.trtri(uch, dch, F)
            s.mark_local_modified(s.origin_slot)
            return int(info.item()) if isinstance(info, torch.Tensor) else int(info)
        # distributed: X = T^{-1} via the distributed trsm against the
        # identity, stored triangle copied back (no gather)
        if dch == 'N':
            z = _first_zero_diag(A)
            if z:
                return z
        X = _general_like(A)
        from .aux import set as aset
        aset(0.0, 1.0, X)
        from .blas3 import trsm
        trsm(Side.Left, 1.0, A, X, opts)
        _copy_tri(X, A)
        return 0


def _general_like(A):
    from ..core.matrix import Matrix
    s = A.storage
    bc = s.bc
    n = A.n()
    X = Matrix(n, n, nb=bc.nb, p=bc.p, q=bc.q, comm=s.comm, dtype=s.dtype, device=s.device, order=bc.order)
    X.insertLocalTiles(device=s.device.index if s.device.type == "cuda" else -1)
    return X


def _first_zero_diag(A):
    """1-based index of the first exactly-zero diagonal element (0: none);
    each rank scans the diagonal runs it owns, one min-reduction."""
    from .aux import _diag_runs
    lb = A.local_block()
    best = 1 << 62
    if lb.mloc and lb.nloc:
        for (i0, j0, k) in _diag_runs(lb.data, lb):
            d = torch.diagonal(lb.data[i0:i0 + k, j0:j0 + k])
            z = (d == 0).nonzero()
            if z.numel():
                best = min(best, lb.global_col(j0 + int(z[0].item())) + 1)
    comm = A.storage.comm
    if comm.size > 1:
        best = int(comm.allreduce_scalar(best, "min", torch.int64))
    return 0 if best >= (1 << 62) else best


def _copy_tri(X, A):
    """Copy the stored triangle of X into triangular A (same distribution:
    one masked local copy, the other triangle of A untouched)."""
    from .aux import copy
    from ..core.matrix import TriangularMatrix as TM
    copy(TM(A.uploPhysical(), X), A)


def trtrm(A, opts=None) -> int:
    """A := L^H L (lower) or U U^H (upper), Hermitian result in the stored
    triangle (LAPACK lauum)."""
    with trace_block("trtrm"):
        s = A.storage
        uplo = A.uploPhysical()
        n = A.n()
        ct = 'C' if s.dtype.is_complex else 'T'
        if _single(A):
            lb = A.local_block()
            F = lb.data[:n, :n]
            big = 1 << 40
            tri = (1 if uplo == Uplo.Lower else 2, big, 1, 0, 1, 0, 0, 0, 0)      # the stored triangle
            other = (2 if uplo == Uplo.Lower else 1, big, 1, 0, 1, 0, 0, 0, -1)   # the rest, strictly
            X = ops.colmajor_empty(n, n, F.dtype, F.device)
            ops.gecopy_mask(F, X, tri)                           # X = tril(F) / triu(F)
            if uplo == Uplo.Lower:
                ops.trmm('L', 'L', ct, 'N', 1.0, F, X)          # X = L^H L
            else:
                ops.trmm('R', 'U', ct, 'N', 1.0, F, X)          # X = U U^H
            # F's stored triangle <- X, its other part unchanged (kernels only)
            W = ops.colmajor_empty(n, n, F.dtype, F.device)
            ops.gecopy_mask(F, W, other)
            ops.gecopy_mask(X, X, tri)
            ops.geadd(1.0, W, 1.0, X)
            F.copy_(X)
            s.mark_local_modified(s.origin_slot)
            return 0
        # distributed: X = stored triangle of A (zeros elsewhere), then the
        # distributed trmm, stored triangle copied back
        X = _general_like(A)
        from .aux import set as aset
        from .blas3 import trmm
        aset(0.0, 0.0, X)
        from ..core.matrix import TriangularMatrix as TM
        from .aux import copy
        copy(TM(uplo, A), TM(uplo, X))
        T = TM(uplo, A, diag=Diag.NonUnit)
        if uplo == Uplo.Lower:
            trmm(Side.Left, 1.0, T.conj_transpose(), X, opts)      # X = L^H L
        else:
            trmm(Side.Right, 1.0, T.conj_transpose(), X, opts)     # X = U U^H
        _copy_tri(X, A)
        return 0
