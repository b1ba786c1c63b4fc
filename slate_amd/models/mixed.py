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


def _mul(alpha, A, X, beta, C, opts):
    """C = alpha A X + beta C with A's structure honoured (hemm for a
    Hermitian A: only its stored triangle is read)."""
    from .blas3 import gemm, hemm
    if isinstance(A, HermitianMatrix):
        return hemm(Side.Left, alpha, A, X, beta, C, opts)
    return gemm(alpha, A, X, beta, C, opts)


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
        _mul(-1.0, A, X, 1.0, R, opts)
        if _converged(R, X, anorm, n):
            return it - 1
        D = solve_lo(R)
        from .aux import add
        add(1.0, D, 1.0, X)
    copy(B, R)
    _mul(-1.0, A, X, 1.0, R, opts)
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
def _col(M, j, j2=None):
    return M.slice(0, M.m() - 1, j, j if j2 is None else j2)


def _small(A, rows, dtype=None):
    """rows x 1 matrix on A's grid (the Hessenberg column / GMRES weights)."""
    s, bc = A.storage, A.storage.bc
    M = Matrix(rows, 1, nb=bc.nb, p=bc.p, q=bc.q, comm=s.comm, dtype=dtype or s.dtype, device=s.device,
               order=bc.order)
    M.insertLocalTiles(device=s.device.index if s.device.type == "cuda" else -1)
    return M


def _givens(f, g):
    """c, s, r with [c s; -conj(s) c] [f; g] = [r; 0] (c real)."""
    import numpy as np
    if g == 0:
        return 1.0, 0.0, f
    if f == 0:
        return 0.0, np.conj(g) / abs(g), abs(g)
    nf, ng = abs(f), abs(g)
    rr = math.hypot(nf, ng)
    c = nf / rr
    sgn = f / nf
    sv = sgn * np.conj(g) / rr
    return c, sv, sgn * rr


def _gmres_ir(A, B, X, precond, opts, anorm):
    """GMRES-based iterative refinement (right-preconditioned restarted
    GMRES on A M^{-1} u = r, M = the low-precision factorization), one
    right-hand side at a time like SLATE (src/gesv_mixed_gmres.cc).  The
    Krylov basis V and the preconditioned vectors Z are distributed n x k
    matrices on A's grid: orthogonalisation is classical Gram-Schmidt with
    one re-orthogonalisation as two GEMMs per pass (V^H w, then w -= V h),
    norms are distributed reductions; only the (restart + 1) x restart
    Hessenberg least-squares problem (Givens rotations) lives on the host,
    as in SLATE."""
    import numpy as np
    from .aux import scale as mscale
    from .blas3 import gemm
    itermax = int(get_option(opts, Option.MaxIterations, 30))
    restart = max(1, min(30, itermax))
    n = A.n()
    dt = B.storage.dtype
    npdt = np.complex128 if dt.is_complex else np.float64
    V = _like(Matrix(n, restart + 1, nb=A.storage.bc.nb, p=A.storage.bc.p, q=A.storage.bc.q, comm=A.storage.comm,
                     dtype=dt, device=A.storage.device, order=A.storage.bc.order), dt)
    Z = _like(V, dt)
    w = _small(A, n, dt)
    total = 0
    for col in range(B.n()):
        Bc, Xc = _col(B, col), _col(X, col)
        for outer in range(max(1, itermax // restart)):
            copy(Bc, w)
            _mul(-1.0, A, Xc, 1.0, w, opts)                      # r = b - A x (working precision)
            if _converged(w, Xc, anorm, n):
                break
            beta = float(norm(Norm.Fro, w))
            if beta == 0:
                break
            v0 = _col(V, 0)
            copy(w, v0)
            mscale(1.0, beta, v0)
            H = np.zeros((restart + 1, restart), dtype=npdt)
            g = np.zeros(restart + 1, dtype=npdt)
            g[0] = beta
            cs, sn = np.zeros(restart), np.zeros(restart, dtype=npdt)
            k = 0
            for j in range(restart):
                precond(_col(V, j), _col(Z, j))                   # z_j = M^{-1} v_j
                _mul(1.0, A, _col(Z, j), 0.0, w, opts)            # w = A z_j
                Vj = _col(V, 0, j)
                hsum = np.zeros(j + 1, dtype=npdt)
                for _ in range(2):                                # CGS2
                    h = _small(A, j + 1, dt)
                    gemm(1.0, Vj.conj_transpose(), w, 0.0, h, opts)
                    gemm(-1.0, Vj, h, 1.0, w, opts)
                    hsum += allgather_dense(h).reshape(-1).cpu().numpy()
                hn = float(norm(Norm.Fro, w))
                H[:j + 1, j] = hsum
                H[j + 1, j] = hn
                for i in range(j):                                 # previous rotations
                    a, b = H[i, j], H[i + 1, j]
                    H[i, j] = cs[i] * a + sn[i] * b
                    H[i + 1, j] = -np.conj(sn[i]) * a + cs[i] * b
                cs[j], sn[j], H[j, j] = _givens(H[j, j], H[j + 1, j])
                H[j + 1, j] = 0
                g[j + 1] = -np.conj(sn[j]) * g[j]
                g[j] = cs[j] * g[j]
                k = j + 1
                total += 1
                if hn == 0 or abs(g[j + 1]) <= 1e-14 * beta:
                    break
                vn = _col(V, j + 1)
                copy(w, vn)
                mscale(1.0, hn, vn)
            # y = R^{-1} g, x += Z y
            y = np.zeros(k, dtype=npdt)
            for i in range(k - 1, -1, -1):
                y[i] = (g[i] - H[i, i + 1:k] @ y[i + 1:k]) / H[i, i]
            Y = _small(A, k, dt)
            from_dense(Y, torch.as_tensor(y.reshape(k, 1)).to(dt))
            gemm(1.0, _col(Z, 0, k - 1), Y, 1.0, Xc, opts)
    return total


def _lo_solve_into(Alo, solve, v, z, lo):
    """z = M^{-1} v with the low-precision factors (distributed copies with
    precision conversion around the solve)."""
    t = _like(v, lo)
    copy(v, t)
    solve(t)
    copy(t, z)


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

        def precond(v, z):
            _lo_solve_into(Alo, lambda t: getrs(Alo, pivots, t, opts), v, z, lo)
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

        def precond(v, z):
            _lo_solve_into(Alo, lambda t: potrs(Alo, t, opts), v, z, lo)
        Xlo = _like(B, lo)
        copy(B, Xlo)
        potrs(Alo, Xlo, opts)
        copy(Xlo, X)
        iters = _gmres_ir(A, B, X, precond, opts, anorm)
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
