"""Condition-number estimation: norm1est (Hager / Higham), gecondest,
pocondest, trcondest.

Reference: `src/gecondest.cc`, `src/pocondest.cc`, `src/trcondest.cc`,
`internal_norm1est.cc` (LAPACK lacn2-style reverse communication with
distributed solves).

MI355X design: the estimator works on distributed n x 1 vectors with the
same row distribution as the factor, and each "apply A^{-1}" / "apply
A^{-H}" is one call of the existing distributed solve (getrs / potrs /
trsm), so all the O(n^2) work stays on the GPUs; only the O(n) vector
reductions (sign, arg-max) are gathered.
"""
from __future__ import annotations

import torch

from ..core.enums import Diag, Norm, Op, Side, Uplo
from ..core.matrix import Matrix, TriangularMatrix
from ..utils.trace import trace_block
from .aux import allgather_dense, from_dense


def _vec_like(A, dtype=None):
    s = A.storage
    bc = s.bc
    n = A.n()
    v = Matrix(n, 1, nb=bc.nb, p=bc.p, q=bc.q, comm=s.comm, dtype=dtype or s.dtype, device=s.device,
               order=bc.order)
    v.insertLocalTiles(device=s.device.index if s.device.type == "cuda" else -1)
    return v


def norm1est(solve, solve_h, n, like):
    """Estimate ||A^{-1}||_1 given x -> A^{-1} x and x -> A^{-H} x acting on
    distributed n x 1 matrices (Higham's refinement of Hager's method)."""
    dt = like.storage.dtype
    cplx = dt.is_complex
    X = _vec_like(like)
    x = torch.full((n, 1), 1.0 / n, dtype=dt)
    est = 0.0
    jlast = -1
    for it in range(5):
        from_dense(X, x)
        solve(X)
        y = allgather_dense(X).cpu()
        ny = float(y.abs().sum())
        if it > 0 and ny <= est:
            break
        est = ny
        xi = torch.where(y.abs() > 0, y / torch.where(y.abs() > 0, y.abs(), torch.ones_like(y.abs())),
                         torch.ones_like(y)) if cplx else torch.where(y >= 0, torch.ones_like(y), -torch.ones_like(y))
        from_dense(X, xi)
        solve_h(X)
        z = allgather_dense(X).cpu()
        j = int(z.abs().argmax())
        if it > 0 and (j == jlast or float(z.abs()[j]) <= float((z.conj() * x).real.sum())):
            break
        jlast = j
        x = torch.zeros((n, 1), dtype=dt)
        x[j] = 1
    # alternating-sign test vector
    alt = torch.tensor([(-1) ** i * (1.0 + i / max(n - 1, 1)) for i in range(n)], dtype=dt).reshape(n, 1)
    from_dense(X, alt)
    solve(X)
    t = 2.0 * float(allgather_dense(X).abs().sum()) / (3.0 * n)
    return max(est, t)


def gecondest(norm_type, A, pivots, anorm, opts=None):
    """Reciprocal condition number of A from its LU factors (getrf)."""
    from .lu import getrs
    with trace_block("gecondest"):
        n = A.n()
        if n == 0:
            return 1.0
        if anorm == 0:
            return 0.0
        nt = Norm.from_string(norm_type) if not isinstance(norm_type, Norm) else norm_type
        fw = (lambda X: getrs(A, pivots, X, opts))
        bw = (lambda X: getrs(A.conj_transpose() if A.storage.dtype.is_complex else A.transpose(), pivots, X, opts))
        if nt == Norm.Inf:
            fw, bw = bw, fw
        ainv = norm1est(fw, bw, n, A)
        return 0.0 if ainv == 0 else 1.0 / (ainv * anorm)


def pocondest(norm_type, A, anorm, opts=None):
    """Reciprocal condition number of the Hermitian positive definite A from
    its Cholesky factor (potrf)."""
    from .chol import potrs
    with trace_block("pocondest"):
        n = A.n()
        if n == 0:
            return 1.0
        if anorm == 0:
            return 0.0
        f = (lambda X: potrs(A, X, opts))
        ainv = norm1est(f, f, n, A)
        return 0.0 if ainv == 0 else 1.0 / (ainv * anorm)


def trcondest(norm_type, A, anorm=None, opts=None):
    """Reciprocal condition number of a triangular matrix."""
    from .blas3 import trsm
    from .aux import norm
    with trace_block("trcondest"):
        n = A.n()
        if n == 0:
            return 1.0
        nt = Norm.from_string(norm_type) if not isinstance(norm_type, Norm) else norm_type
        if anorm is None:
            anorm = float(norm(nt, A, opts))
        if anorm == 0:
            return 0.0
        fw = (lambda X: trsm(Side.Left, 1.0, A, X, opts))
        Ah = A.conj_transpose() if A.storage.dtype.is_complex else A.transpose()
        bw = (lambda X: trsm(Side.Left, 1.0, Ah, X, opts))
        if nt == Norm.Inf:
            fw, bw = bw, fw
        ainv = norm1est(fw, bw, n, A)
        return 0.0 if ainv == 0 else 1.0 / (ainv * anorm)
