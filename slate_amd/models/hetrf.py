"""Symmetric/Hermitian indefinite solvers: hetrf / hetrs / hesv (and the
sy* aliases) -- P A P^H = L T L^H with T Hermitian tridiagonal.

Reference: `src/hetrf.cc` (blocked Aasen, host only: "GPU version not yet
implemented", `src/hetrf.cc:23`; band T factored by gbtrf, `:511`),
`src/hetrs.cc:94-105` (trsm + gbtrs + trsm), `src/hesv.cc`.

MI355X design: the factorization runs on the GPU as the Parlett-Reid
elimination (same L T L^H form as Aasen, partial pivoting on the
subdiagonal column): one rank-2 two-sided update of the trailing matrix
per column, expressed as device tensor kernels with the pivot index kept
ON the device (no host synchronisation per column).  T is then factored by
a pivoted tridiagonal LU (gtsv) and the solve is two triangular solves
around it.  Distributed matrices are gathered (the factorization is O(n^3)
on one GPU; SLATE's hetrf is host-only).
"""
from __future__ import annotations

import torch

from .. import ops
from ..core.enums import Uplo
from ..core.matrix import Pivots
from ..utils.trace import trace_block
from .aux import allgather_dense, from_dense


class IndefiniteFactors:
    def __init__(self, L, d, e, perm):
        self.L, self.d, self.e, self.perm = L, d, e, perm


def _full(A):
    from .eig import _dense_hermitian
    return _dense_hermitian(A)


def hetrf(A, pivots: Pivots = None, T=None, pivots2=None, H=None, opts=None):
    """Factor the Hermitian indefinite A: P A P^H = L T L^H.  L (unit lower,
    first column e1) overwrites the lower triangle of A below the
    subdiagonal; T is returned (and written into the band matrix T if
    given); the permutation goes to `pivots`.  Returns info (0)."""
    with trace_block("hetrf"):
        W = _full(A).clone()
        n = W.shape[0]
        dev = W.device
        perm = torch.arange(n, device=dev)
        Lm = torch.eye(n, dtype=W.dtype, device=dev)
        for k in range(n - 2):
            col = W[k + 1:, k].abs()
            p = k + 1 + torch.argmax(col)                     # device scalar: no host sync
            # symmetric swap of rows/cols k+1 <-> p (and L rows, perm)
            idx = torch.stack([torch.tensor(k + 1, device=dev), p])
            rev = idx.flip(0)
            W[idx] = W[rev]
            W[:, idx] = W[:, rev]
            perm[idx] = perm[rev]
            Lm[idx, :k + 1] = Lm[rev, :k + 1]
            piv = W[k + 1, k]
            safe = torch.where(piv == 0, torch.ones_like(piv), piv)
            l = torch.where(piv == 0, torch.zeros_like(W[k + 2:, k]), W[k + 2:, k] / safe)
            Lm[k + 2:, k + 1] = l
            # two-sided Gauss transform: rows then columns
            W[k + 2:, k:] -= l[:, None] * W[k + 1, k:][None, :]
            W[k:, k + 2:] -= W[k:, k + 1][:, None] * l.conj()[None, :]
        d = torch.diagonal(W).real.clone() if W.is_complex() else torch.diagonal(W).clone()
        e = torch.diagonal(W, -1).clone()
        F = IndefiniteFactors(Lm, d, e, perm)
        # store L below the subdiagonal of A (SLATE keeps L in A)
        Ad = allgather_dense(A)
        up = A.uploPhysical()
        # LAPACK sytrf_aa-like layout: T on the diagonal/subdiagonal, L(:, 1:)
        # shifted one column left below the subdiagonal
        Lsh = torch.zeros_like(Lm)
        if n > 1:
            Lsh[:, :n - 1] = torch.tril(Lm[:, 1:], -2)
        out = Lsh + torch.diag(torch.diagonal(W)) + torch.diag(e, -1)
        if up == Uplo.Upper:
            out = out.mH
        from_dense(A, out.to(Ad.dtype))
        A._hetrf = F
        if pivots is not None:
            pivots.set(perm.to(torch.int64), 1)
        if T is not None:
            from_dense(T, (torch.diag(torch.diagonal(W)) + torch.diag(e, -1) + torch.diag(e.conj(), 1)).to(Ad.dtype))
        return 0


def _gtsv(d, e, B):
    """Solve the Hermitian tridiagonal T X = B (T: diag d, subdiag e) by LU
    with partial pivoting (host, O(n nrhs))."""
    n = d.numel()
    dt = B.dtype
    dl = e.to(dt).cpu().clone()
    du = e.conj().to(dt).cpu().clone()
    dd = d.to(dt).cpu().clone()
    du2 = torch.zeros(max(n - 2, 0), dtype=dt)
    X = B.cpu().clone()
    ipv = list(range(n))
    for i in range(n - 1):
        if abs(dd[i]) >= abs(dl[i]):
            if dd[i] == 0:
                raise ZeroDivisionError("singular tridiagonal")
            f = dl[i] / dd[i]
            dd[i + 1] -= f * du[i]
            X[i + 1] -= f * X[i]
            if i < n - 2:
                du2[i] = 0
        else:
            f = dd[i] / dl[i]
            dd[i], dl[i] = dl[i], dd[i]
            tmp = du[i].clone()
            du[i] = dd[i + 1]
            dd[i + 1] = tmp - f * dd[i + 1]
            if i < n - 2:
                du2[i] = du[i + 1]
                du[i + 1] = -f * du[i + 1]
            Xi = X[i].clone()
            X[i] = X[i + 1]
            X[i + 1] = Xi - f * X[i + 1]
            dl[i] = f
    # back substitution
    X[n - 1] /= dd[n - 1]
    if n > 1:
        X[n - 2] = (X[n - 2] - du[n - 2] * X[n - 1]) / dd[n - 2]
    for i in range(n - 3, -1, -1):
        X[i] = (X[i] - du[i] * X[i + 1] - du2[i] * X[i + 2]) / dd[i]
    return X


def hetrs(A, pivots=None, T=None, pivots2=None, B=None, opts=None):
    """Solve A X = B with the factors of hetrf (B overwritten)."""
    with trace_block("hetrs"):
        F = A._hetrf
        Bd = allgather_dense(B)
        dev = F.L.device
        Y = Bd.to(dev)[F.perm]
        Lc = ops.as_colmajor(F.L.clone())
        Yc = ops.as_colmajor(Y.clone())
        ops.trsm('L', 'L', 'N', 'U', 1.0, Lc, Yc)
        Z = _gtsv(F.d, F.e, Yc).to(dev)
        Zc = ops.as_colmajor(Z.clone())
        ops.trsm('L', 'L', 'C' if Zc.is_complex() else 'T', 'U', 1.0, Lc, Zc)
        X = torch.empty_like(Zc)
        X[F.perm] = Zc
        from_dense(B, X.to(Bd.dtype))
        return 0


def hesv(A, pivots=None, T=None, pivots2=None, H=None, B=None, opts=None) -> int:
    info = hetrf(A, pivots, T, pivots2, H, opts)
    if info == 0:
        hetrs(A, pivots, T, pivots2, B, opts)
    return info


sytrf = hetrf
sytrs = hetrs
sysv = hesv
