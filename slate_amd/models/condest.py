"""Condition-number estimation: norm1est (Hager / Higham), gecondest,
pocondest, trcondest.

Reference: `src/gecondest.cc`, `src/pocondest.cc`, `src/trcondest.cc`,
`internal_norm1est.cc` (LAPACK lacn2-style reverse communication with
distributed solves).

MI355X design: the estimator works on distributed n x 1 vectors with the
same row distribution as the factor, and each "apply A^{-1}" / "apply
A^{-H}" is one call of the existing distributed solve (getrs / potrs /
trsm), so all the O(n^2) work stays on the GPUs; the O(n) vector steps
run on each rank's local part with scalar reductions only.
"""
from __future__ import annotations

import torch

from ..core.enums import Diag, Norm, Op, Side, Uplo
from ..core.matrix import Matrix, TriangularMatrix
from .. import ops
from ..utils.trace import trace_block


def _vec_like(A, dtype=None):
    s = A.storage
    bc = s.bc
    n = A.n()
    v = Matrix(n, 1, nb=bc.nb, p=bc.p, q=bc.q, comm=s.comm, dtype=dtype or s.dtype, device=s.device,
               order=bc.order)
    v.insertLocalTiles(device=s.device.index if s.device.type == "cuda" else -1)
    return v


class _DistVec:
    """This rank's part of a distributed n x 1 vector X (the local rows and
    their global indices): the estimator's O(n) vector operations run on
    the local parts, with scalar reductions only."""

    def __init__(self, X):
        self.X = X
        lb = X.local_block()
        self.lb = lb
        self.comm = X.storage.comm
        self.owner = lb.nloc > 0 and lb.mloc > 0
        self.rows = torch.as_tensor([lb.global_row(i) for i in range(lb.mloc)], dtype=torch.int64) \
            if self.owner else torch.zeros(0, dtype=torch.int64)

    @property
    def v(self):
        return self.lb.data[:self.lb.mloc, 0] if self.owner else None

    @property
    def col(self):
        """the local part as a column-major mloc x 1 block (kernel operand)"""
        return self.lb.data[:self.lb.mloc, :1] if self.owner else None

    def fill(self, fn):
        """v[i] = fn(global index tensor) (host values)."""
        if self.owner:
            self.v.copy_(fn(self.rows).to(self.v.dtype).to(self.v.device))
        self.X.storage.mark_local_modified(self.X.storage.origin_slot)

    def sum_abs(self):
        loc = float(ops.genorm_local('1', self.col)[0][0]) if self.owner else 0.0
        return self.comm.allreduce_scalar(loc) if self.comm.size > 1 else loc

    def argmax_abs(self):
        if self.owner and self.v.numel():
            a = self.v.abs()
            i = int(a.argmax())
            val, idx = float(a[i]), int(self.rows[i])
        else:
            val, idx = -1.0, 1 << 62
        return self.comm.maxloc(val, idx) if self.comm.size > 1 else (val, idx)

    def dot_real(self, fn_x):
        """sum_i real(conj(v_i) x_i) with x given by its global-index function."""
        loc = 0.0
        if self.owner:
            x = fn_x(self.rows).to(self.v.dtype).to(self.v.device).view(-1, 1)
            d = torch.zeros(1, 1, dtype=self.v.dtype, device=self.v.device)
            ops.gemm(1.0, self.col, x, 0.0, d, transA='C')       # v^H x
            loc = float(d[0, 0].real)
        return self.comm.allreduce_scalar(loc) if self.comm.size > 1 else loc

    def to_sign(self):
        """v := v / |v| (1 where v = 0), in place on the local part."""
        if self.owner and self.v.numel():
            ops.gescale_row_col('S', None, None, self.col)
        self.X.storage.mark_local_modified(self.X.storage.origin_slot)


def norm1est(solve, solve_h, n, like):
    """Estimate ||A^{-1}||_1 given X -> A^{-1} X and X -> A^{-H} X acting on
    distributed n x 1 matrices (Higham's refinement of Hager's method,
    LAPACK lacn2).  The vectors never leave their ranks: 1-norms, the
    sign vector, the arg-max and the dot products are local operations
    plus scalar reductions (SLATE internal_norm1est.cc: MPI_Bcast of
    isave/kase/est and an MPI_Allreduce MAXLOC)."""
    X = _vec_like(like)
    V = _DistVec(X)
    V.fill(lambda g: torch.full((g.numel(),), 1.0 / n, dtype=torch.float64))
    xfn = lambda g: torch.full((g.numel(),), 1.0 / n, dtype=torch.float64)   # noqa: E731
    est = 0.0
    jlast = -1
    for it in range(5):
        solve(X)
        V = _DistVec(X)
        ny = V.sum_abs()
        if it > 0 and ny <= est:
            break
        est = ny
        V.to_sign()
        solve_h(X)
        V = _DistVec(X)
        zj, j = V.argmax_abs()
        if it > 0 and (j == jlast or zj <= V.dot_real(xfn)):
            break
        jlast = j
        xfn = (lambda jj: (lambda g: (g == jj).to(torch.float64)))(j)
        V.fill(xfn)
    # alternating-sign test vector
    V = _DistVec(X)
    V.fill(lambda g: torch.where(g % 2 == 0, 1.0, -1.0).to(torch.float64) * (1.0 + g.to(torch.float64) /
                                                                              max(n - 1, 1)))
    solve(X)
    t = 2.0 * _DistVec(X).sum_abs() / (3.0 * n)
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
