"""Mixed-precision solvers and random butterfly transforms: gesv_mixed,
posv_mixed (low-precision factor + high-precision iterative refinement),
gesv_mixed_gmres, posv_mixed_gmres (GMRES-IR), gerbt, gesv_rbt.

Reference: `src/gesv_mixed.cc:105-290`, `src/posv_mixed.cc`,
`src/gesv_mixed_gmres.cc`, `src/posv_mixed_gmres.cc`, `src/gesv_rbt.cc`,
`src/gerbt.cc`, `internal_gerbt.cc`, `internal_rbt_generate.cc`.

MI355X design: the factorization runs in fp32 (the gfx950 fp32 MFMA path,
2x the fp64 rate) on the same block-cyclic layout (one gecopy kernel per
rank converts), the residual GEMM in fp64; everything stays on the GPUs,
only scalars (norms, convergence) reach the host.  The RBT is applied to
the whole matrix as two recursive butterfly sweeps with random diagonal
scalings from the counter-based Philox stream (reproducible across grids).
"""
from __future__ import annotations

import math

import torch

from .. import ops
from ..core.enums import Diag, Norm, Op, Option, Side, Uplo
from ..core.exceptions import SlateError
from ..core.matrix import HermitianMatrix, Matrix, Pivots, TriangularMatrix
from ..core.options import get_option
from ..utils.trace import trace_block
from .aux import allgather_dense, copy, from_dense, norm


def _lo_dtype(dt):
    return {torch.float64: torch.float32, torch.complex128: torch.complex64}.get(dt, dt)


def _like(A, dtype=None, cls=Matrix, **kw):
    s = A.storage
    bc = s.bc
    if cls is HermitianMatrix:
        M = HermitianMatrix(A.uploPhysical(), A.n(), nb=bc.nb, p=bc.p, q=bc.q, comm=s.comm,
                            dtype=dtype or s.dtype, device=s.device)
    else:
        M = Matrix(A.m(), A.n(), nb=bc.nb, p=bc.p, q=bc.q, comm=s.comm, dtype=dtype or s.dtype,
                   device=s.device, order=bc.order)
    M.insertLocalTiles(device=s.device.index if s.device.type == "cuda" else -1)
    return M


def _converged(R, X, anorm, n):
    """Column-wise test of iterRefConverged (src/internal/internal_util.hh:121-136):
    max|R_j| <= max|X_j| * ||A||_inf * eps * sqrt(n) for EVERY right-hand side j."""
    from .aux import colNorms
    eps = torch.finfo(torch.float64).eps
    cte = anorm * eps * math.sqrt(n)
    rn = colNorms(Norm.Max, R)
    xn = colNorms(Norm.Max, X)
    if torch.isnan(rn).any() or torch.isnan(xn).any():
        return False
    return bool((rn <= xn * cte).all())


def _fallback(solver, args, B, X, opts, info_lo):
    """Low-precision factorization failed (info_lo > 0): with
    Option.UseFallbackSolver (default) solve in full precision into X and
    report iter = -3 like SLATE; otherwise return the low-precision info."""
    if not get_option(opts, Option.UseFallbackSolver, True):
        return info_lo, -3
    copy(B, X)
    info = solver(*args, X, opts)
    return info, -3


def _refine(A, B, X, solve_lo, opts, anorm):
    """Classic IR: X += solve_lo(B - A X) until converged; returns iters (<0
    if not converged)."""
    from .blas3 import gemm
    itermax = int(get_option(opts, Option.MaxIterations, 30))
    n = A.n()
    R = _like(B)
    for it in range(1, itermax + 1):
        copy(B, R)
        gemm(-1.0, A, X, 1.0, R, opts)
        if _converged(R, X, anorm, n):
            return it - 1
        D = solve_lo(R)
        from .aux import add
        add(1.0, D, 1.0, X)
    copy(B, R)
    gemm(-1.0, A, X, 1.0, R, opts)
    return itermax if _converged(R, X, anorm, n) else -itermax


def gesv_mixed(A, pivots, B, X, opts=None):
    """Solve A X = B: fp32 LU + fp64 iterative refinement.  Returns
    (info, iters); falls back to fp64 gesv if IR does not converge and
    Option.UseFallbackSolver (default True)."""
    from .lu import getrf, getrs, gesv
    with trace_block("gesv_mixed"):
        lo = _lo_dtype(A.storage.dtype)
        Alo = _like(A, lo)
        copy(A, Alo)
        info = getrf(Alo, pivots, opts)
        if info:
            # the fp32 factor is singular although A may not be: iter = -3 and
            # refactor in full precision (src/gesv_mixed.cc:185-187, 256-277)
            return _fallback(gesv, (A, pivots), B, X, opts, info)
        anorm = float(norm(Norm.Inf, A))

        def solve_lo(R):
            Rlo = _like(R, lo)
            copy(R, Rlo)
            getrs(Alo, pivots, Rlo, opts)
            D = _like(R)
            copy(Rlo, D)
            return D
        Xi = solve_lo(B)
        copy(Xi, X)
        iters = _refine(A, B, X, solve_lo, opts, anorm)
        if iters < 0 and get_option(opts, Option.UseFallbackSolver, True):
            copy(B, X)
            info = gesv(A, pivots, X, opts)
        return info, iters


def posv_mixed(A, B, X, opts=None):
    """Hermitian positive definite A X = B: fp32 Cholesky + fp64 IR."""
    from .chol import potrf, potrs, posv
    with trace_block("posv_mixed"):
        lo = _lo_dtype(A.storage.dtype)
        Alo = _like(A, lo, HermitianMatrix)
        copy(A, Alo)
        info = potrf(Alo, opts)
        if info:
            return _fallback(posv, (A,), B, X, opts, info)
        anorm = float(norm(Norm.Inf, A))

        def solve_lo(R):
            Rlo = _like(R, lo)
            copy(R, Rlo)
            potrs(Alo, Rlo, opts)
            D = _like(R)
            copy(Rlo, D)
            return D
        copy(solve_lo(B), X)
        iters = _refine(A, B, X, solve_lo, opts, anorm)
        if iters < 0 and get_option(opts, Option.UseFallbackSolver, True):
            copy(B, X)
            info = posv(A, X, opts)
        return info, iters


# ------------------------------------------------------------------ GMRES-IR
def _gmres_ir(A, B, X, precond, opts, anorm):
    """GMRES-based iterative refinement (right-preconditioned restarted
    GMRES on A M^{-1} u = r, M = low-precision factorization), one RHS at a
    time like SLATE (src/gesv_mixed_gmres.cc)."""
    from .blas3 import gemm
    itermax = int(get_option(opts, Option.MaxIterations, 30))
    restart = min(30, itermax)
    n = A.n()
    Xd = allgather_dense(X)
    Bd = allgather_dense(B)
    dev = Xd.device
    total = 0
    R = _like(B)
    for col in range(B.n()):
        for outer in range(max(1, itermax // max(restart, 1))):
            # residual r = b - A x (fp64, distributed)
            copy(B, R)
            gemm(-1.0, A, X, 1.0, R, opts)
            Rd = allgather_dense(R)[:, col]
            Xc = allgather_dense(X)
            if float(Rd.abs().max()) <= float(Xc[:, col].abs().max()) * anorm * torch.finfo(torch.float64).eps * \
                    math.sqrt(n):
                break
            beta = float(torch.linalg.vector_norm(Rd))
            if beta == 0:
                break
            Vb = [Rd / beta]
            Hm = torch.zeros(restart + 1, restart, dtype=Rd.dtype)
            g = torch.zeros(restart + 1, dtype=Rd.dtype)
            g[0] = beta
            Zs = []
            k_used = 0
            for j in range(restart):
                z = precond(Vb[j])                     # z = M^{-1} v
                Zs.append(z)
                w = _matvec(A, z, opts)                # w = A z
                for i in range(j + 1):
                    Hm[i, j] = torch.dot(Vb[i].conj(), w).item()
                    w = w - Hm[i, j] * Vb[i]
                Hm[j + 1, j] = torch.linalg.vector_norm(w).item()
                k_used = j + 1
                total += 1
                # least-squares residual estimate
                y = torch.linalg.lstsq(Hm[:j + 2, :j + 1], g[:j + 2, None]).solution
                res = torch.linalg.vector_norm(Hm[:j + 2, :j + 1] @ y - g[:j + 2, None])
                if float(Hm[j + 1, j]) == 0 or float(res) <= 1e-14 * beta:
                    break
                Vb.append(w / Hm[j + 1, j])
            y = torch.linalg.lstsq(Hm[:k_used + 1, :k_used], g[:k_used + 1, None]).solution.reshape(-1)
            upd = sum(y[i] * Zs[i] for i in range(k_used))
            Xc[:, col] = Xc[:, col] + upd
            from_dense(X, Xc)
    return total


def _matvec(A, z, opts):
    from .blas3 import gemm
    Z = _vec(A, z)
    W = _vec(A, torch.zeros_like(z))
    gemm(1.0, A, Z, 0.0, W, opts)
    return allgather_dense(W)[:, 0]


def _vec(A, v):
    s = A.storage
    bc = s.bc
    V = Matrix(A.n(), 1, nb=bc.nb, p=bc.p, q=bc.q, comm=s.comm, dtype=v.dtype, device=s.device, order=bc.order)
    V.insertLocalTiles(device=s.device.index if s.device.type == "cuda" else -1)
    from_dense(V, v.reshape(-1, 1))
    return V


def gesv_mixed_gmres(A, pivots, B, X, opts=None):
    from .lu import getrf, getrs, gesv
    with trace_block("gesv_mixed_gmres"):
        lo = _lo_dtype(A.storage.dtype)
        Alo = _like(A, lo)
        copy(A, Alo)
        info = getrf(Alo, pivots, opts)
        if info:
            return _fallback(gesv, (A, pivots), B, X, opts, info)
        anorm = float(norm(Norm.Inf, A))

        def precond(v):
            V = _vec(Alo, v.to(lo))
            getrs(Alo, pivots, V, opts)
            return allgather_dense(V)[:, 0].to(v.dtype)
        Xlo = _like(B, lo)
        copy(B, Xlo)
        getrs(Alo, pivots, Xlo, opts)
        copy(Xlo, X)
        iters = _gmres_ir(A, B, X, precond, opts, anorm)
        return info, iters


def posv_mixed_gmres(A, B, X, opts=None):
    from .chol import potrf, potrs, posv
    with trace_block("posv_mixed_gmres"):
        lo = _lo_dtype(A.storage.dtype)
        Alo = _like(A, lo, HermitianMatrix)
        copy(A, Alo)
        info = potrf(Alo, opts)
        if info:
            return _fallback(posv, (A,), B, X, opts, info)
        anorm = float(norm(Norm.Inf, A))

        def precond(v):
            V = _vec(Alo, v.to(lo))
            potrs(Alo, V, opts)
            return allgather_dense(V)[:, 0].to(v.dtype)
        Xlo = _like(B, lo)
        copy(B, Xlo)
        potrs(Alo, Xlo, opts)
        copy(Xlo, X)
        Ah = A
        iters = _gmres_ir(Ah, B, X, precond, opts, anorm)
        return info, iters


# ------------------------------------------------------------------ RBT
def _butterfly_diag(n, depth, seed, dtype=torch.float64, device="cpu"):
    """Random diagonals of the recursive butterflies (depth levels):
    entries exp(r / 10), r uniform in [-1/2, 1/2) (Baboulin et al.)."""
    g = torch.Generator().manual_seed(int(seed))
    r = torch.rand(depth, n, generator=g, dtype=torch.float64) - 0.5
    return torch.exp(r / 10.0).to(dtype).to(device)


def rbt_size(n, depth, nb, p=1, q=1):
    """Order the butterflies act on: n padded to a multiple of
    2^depth nb lcm(p, q).  Then every butterfly partner (global distance
    >= N / 2^depth, a multiple of nb p and nb q) lies on the SAME process
    row / column, at local distance (global distance) / p (or / q): the
    transform is a purely local kernel on every rank, no communication
    (SLATE pairs tiles across ranks with tile sends, internal_gerbt.cc)."""
    unit = (1 << depth) * nb * (p * q // math.gcd(p, q))
    return max(unit, -(-n // unit) * unit)


class Butterfly:
    """W = W_depth ... W_1 of order N (the RBT factor U or V); ``diag``
    (depth x N host fp64) holds the random diagonals."""

    def __init__(self, N, depth, seed):
        self.N, self.depth = N, depth
        self.diag = _butterfly_diag(N, depth, seed)

    def local(self, rows_global, dtype, device):
        rdt = torch.float32 if dtype in (torch.float32, torch.complex64) else torch.float64
        d = self.diag[:, rows_global] if rows_global is not None else self.diag
        return d.to(rdt).contiguous().to(device)


def _local_index(M, dim):
    lb = M.local_block()
    if dim == 'row':
        return lb, torch.as_tensor([lb.global_row(i) for i in range(lb.mloc)], dtype=torch.int64)
    return lb, torch.as_tensor([lb.global_col(j) for j in range(lb.nloc)], dtype=torch.int64)


def _apply_w(W: Butterfly, M, trans, side):
    """M := op(W) M (side 'L', on M's rows) or M op(W)^T (side 'R', on M's
    column index), op(W) = W^T when ``trans``; locally on every rank (see
    rbt_size)."""
    s = M.storage
    if s.bc is None:
        raise SlateError("RBT needs a block-cyclic matrix")
    lb, idx = _local_index(M, 'row' if side == 'L' else 'col')
    if idx.numel() == 0 or (lb.mloc == 0 or lb.nloc == 0):
        return
    X = lb.data[:lb.mloc, :lb.nloc]
    ops.butterfly(X, W.local(idx, s.dtype, X.device), W.depth, trans, side)
    s.mark_local_modified(s.origin_slot)


def gerbt(U, A, V):
    """A := U^T A V in place (SLATE gerbt(U, A, V), src/gerbt.cc); U, V are
    :class:`Butterfly` of A's order (a multiple of rbt_size's unit)."""
    with trace_block("gerbt"):
        _apply_w(U, A, True, 'L')         # U^T A
        _apply_w(V, A, True, 'R')         # (U^T A) V = (U^T A) (W^T)^T
    return A


def _padded(M, N, ncols=None, identity=False):
    """N x ncols copy of M (zero padding; identity on the padded diagonal)."""
    from .aux import set as aset
    s, bc = M.storage, M.storage.bc
    ncols = N if ncols is None else ncols
    Pm = Matrix(N, ncols, nb=bc.nb, p=bc.p, q=bc.q, comm=s.comm, dtype=s.dtype, device=s.device, order=bc.order)
    Pm.insertLocalTiles(device=s.device.index if s.device.type == "cuda" else -1)
    aset(0.0, 1.0 if identity else 0.0, Pm)
    copy(M, Pm.slice(0, M.m() - 1, 0, M.n() - 1))
    return Pm


def gesv_rbt(A, B, opts=None):
    """Solve A X = B with a random butterfly transform + LU without pivoting
    + iterative refinement in working precision (src/gesv_rbt.cc).  A is
    embedded in diag(A, I) of the padded order when n is not a multiple of
    rbt_size's unit (no silent switch to partial pivoting)."""
    from .lu import getrf_nopiv, getrs_nopiv
    with trace_block("gesv_rbt"):
        depth = max(1, min(4, int(get_option(opts, Option.Depth, 2))))
        n = A.n()
        bc = A.storage.bc
        if bc is None:
            from .aux import run_on_block_cyclic
            return run_on_block_cyclic(A, lambda Ab, o: gesv_rbt(Ab, B, o), opts)
        N = rbt_size(n, depth, bc.nb, bc.p, bc.q)
        A0 = _like(A)
        copy(A, A0)
        Ap = A if N == n else _padded(A, N, identity=True)
        U = Butterfly(N, depth, 7)
        V = Butterfly(N, depth, 8)
        gerbt(U, Ap, V)
        info = getrf_nopiv(Ap, opts)
        if info:
            return info
        anorm = float(norm(Norm.Inf, A0))

        def solve(R):
            # x = V (LU)^{-1} U^T r  (on the padded order)
            Y = _padded(R, N, R.n())
            _apply_w(U, Y, True, 'L')
            getrs_nopiv(Ap, Y, opts)
            _apply_w(V, Y, False, 'L')
            D = _like(R)
            copy(Y.slice(0, n - 1, 0, R.n() - 1), D)
            return D
        X = solve(B)
        _refine(A0, B, X, solve, {**(opts or {}), Option.MaxIterations: int(get_option(opts, Option.MaxIterations,
                                                                                       10))}, anorm)
        copy(X, B)
        return 0
