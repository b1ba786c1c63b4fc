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
def _butterfly_diag(n, depth, seed, dtype, device):
    """Random diagonals of the recursive butterflies (depth levels):
    entries exp(r / 10), r uniform in [-1/2, 1/2) (Baboulin et al.)."""
    g = torch.Generator().manual_seed(int(seed))
    r = torch.rand(depth, n, generator=g, dtype=torch.float64) - 0.5
    return torch.exp(r / 10.0).to(dtype).to(device)


def _apply_butterfly(D, diags, trans, side):
    """Apply W = W_depth ... W_1 (each level block-diagonal with 2^l
    butterflies [R0 R1; R0 -R1]/sqrt 2) to the rows (side 'L') or columns
    ('R') of dense D in place; trans applies W^T."""
    n = D.shape[0] if side == 'L' else D.shape[1]
    depth = diags.shape[0]
    X = D if side == 'L' else D.transpose(0, 1)
    levels = range(depth) if not trans else range(depth - 1, -1, -1)
    for lvl in levels:
        nblk = 2 ** lvl
        size = n // nblk
        if size < 2:
            continue
        h = size // 2
        for b in range(nblk):
            o = b * size
            r0 = diags[lvl, o:o + h][:, None]
            r1 = diags[lvl, o + h:o + 2 * h][:, None]
            top = X[o:o + h].clone()
            bot = X[o + h:o + 2 * h].clone()
            s = 1.0 / math.sqrt(2.0)
            if not trans:
                # [R0 R1; R0 -R1] / sqrt 2  applied to [top; bot]
                X[o:o + h] = s * (r0 * top + r1 * bot)
                X[o + h:o + 2 * h] = s * (r0 * top - r1 * bot)
            else:
                # transpose: [R0 R0; R1 -R1] / sqrt 2
                X[o:o + h] = s * r0 * (top + bot)
                X[o + h:o + 2 * h] = s * r1 * (top - bot)
    return D


def gerbt(U, A, V, depth=2, seed=7):
    """A := U^T A V with random butterflies (returned diagonals (du, dv))."""
    D = allgather_dense(A).clone()
    n = D.shape[0]
    du = _butterfly_diag(n, depth, seed, D.dtype, D.device)
    dv = _butterfly_diag(n, depth, seed + 1, D.dtype, D.device)
    _apply_butterfly(D, du, True, 'L')        # U^T A
    _apply_butterfly(D, dv, True, 'R')        # (U^T A) V : columns
    from_dense(A, D)
    return du, dv


def gesv_rbt(A, B, opts=None):
    """Solve A X = B with a random butterfly transform + LU without pivoting
    + iterative refinement in working precision (src/gesv_rbt.cc)."""
    from .lu import getrf_nopiv, getrs_nopiv, gesv
    with trace_block("gesv_rbt"):
        depth = int(get_option(opts, Option.Depth, 2))
        n = A.n()
        pad = (1 << depth)
        if n % pad:
            # butterflies need n divisible by 2^depth: partial pivoting instead
            from ..core.enums import MethodLU
            o = dict(opts or {})
            o[Option.MethodLU] = MethodLU.PartialPiv
            return gesv(A, Pivots(), B, o)
        A0 = _like(A)
        copy(A, A0)
        du, dv = gerbt(None, A, None, depth)
        info = getrf_nopiv(A, opts)
        if info:
            return info
        anorm = float(norm(Norm.Inf, A0))

        def solve(R):
            # x = V (LU)^{-1} U^T r
            Rd = allgather_dense(R).clone()
            _apply_butterfly(Rd, du, True, 'L')
            Y = _like(R)
            from_dense(Y, Rd)
            getrs_nopiv(A, Y, opts)
            Yd = allgather_dense(Y).clone()
            _apply_butterfly(Yd, dv, False, 'L')
            from_dense(Y, Yd)
            return Y
        X = solve(B)
        _refine(A0, B, X, solve, {**(opts or {}), Option.MaxIterations: int(get_option(opts, Option.MaxIterations,
                                                                                       10))}, anorm)
        copy(X, B)
        return 0
