"""Tile/block-level compute operations on column-major tensor views.

Each function dispatches by where the data lives: tensors on the MI355X go
to the gfx950 kernels in ``_hip`` (MFMA GEMM, tile potrf, blocked trsm,
GPU LU panel, row permutations, norms, ...), host tensors go to the native
C++ kernels in ``_host``.  There is no PyTorch/vendor-library fallback: a
missing ``_hip`` raises.  All device calls are enqueued on the CURRENT
torch stream (so callers express overlap with ``torch.cuda.stream(...)``)
and never synchronise the host.

Conventions (LAPACK/SLATE): matrices are 2-D views with ``stride(0) == 1``
(column-major); ``trans`` is 'N'/'T'/'C'; ``uplo`` 'L'/'U'/'G';
pivots are 0-based int64 row indices.
"""
from __future__ import annotations

import torch

from .. import _native
from .._native import code, kmod, stream
from ..core.exceptions import SlateError

_WORK = {}
_FLOPS = None     # [count] while a flop_counter() is active


class flop_counter:
    """Count the multiply-add flops the BLAS-3 ops of this process issue
    (2 m n k per GEMM, m^2 n per triangular multiply / solve), e.g. to check
    that a distributed trmm does the triangular, not the dense, count."""

    def __enter__(self):
        global _FLOPS
        self._prev, _FLOPS = _FLOPS, [0]
        return self

    def __exit__(self, *exc):
        global _FLOPS
        self.flops = _FLOPS[0]
        _FLOPS = self._prev
        return False


def _chk(t: torch.Tensor, name="A"):
    if t.dim() != 2:
        raise SlateError(f"{name} must be 2-D")
    if t.shape[0] > 1 and t.shape[1] > 0 and t.stride(0) != 1:
        raise SlateError(f"{name} must be column-major (stride(0)==1), got strides {t.stride()}")


def ld(t: torch.Tensor) -> int:
    return max(1, t.stride(1), t.shape[0]) if t.shape[1] <= 1 else max(1, t.stride(1))


def _c(x):
    return complex(x)


def _ch(x):
    """normalise enum/str arguments to the kernels' char codes"""
    return str(x)[0] if not hasattr(x, "value") else x.value


def colmajor_empty(m, n, dtype, device):
    return torch.empty((n, max(m, 1)), dtype=dtype, device=device).t()[:m, :]


def colmajor_zeros(m, n, dtype, device):
    return torch.zeros((n, max(m, 1)), dtype=dtype, device=device).t()[:m, :]


def as_colmajor(t: torch.Tensor) -> torch.Tensor:
    """Column-major copy/view of a 2-D tensor."""
    if t.dim() == 2 and (t.stride(0) == 1 or t.shape[0] <= 1):
        return t
    return t.t().contiguous().t()


# ----------------------------------------------------------------- BLAS 3
def gemm(alpha, A, B, beta, C, transA='N', transB='N', mask=None, batch=1, strides=(0, 0, 0)):
    """C = alpha op(A) op(B) + beta C  (one MFMA launch on device)."""
    _chk(C, "C")
    m, n = C.shape
    if m == 0 or n == 0:
        return C
    ta, tb = _ch(transA), _ch(transB)
    k = A.shape[1] if ta == 'N' else A.shape[0]
    if k == 0 or alpha == 0:
        if beta != 1:
            gescale(beta, C)
        return C
    _chk(A, "A"); _chk(B, "B")
    if _FLOPS is not None:
        _FLOPS[0] += 2 * m * n * k * max(1, batch)
    kmod(C).gemm(code(C.dtype), ta, tb, m, n, k, _c(alpha), A.data_ptr(), ld(A), B.data_ptr(), ld(B),
                 _c(beta), C.data_ptr(), ld(C), batch, strides[0], strides[1], strides[2], mask, stream(C))
    return C


def herk(uplo, trans, alpha, A, beta, C, mask=None):
    """C = alpha A A^H + beta C (trans='N') or alpha A^H A + beta C; only the
    `uplo` triangle of C is written (TriMask inside the GEMM epilogue)."""
    cplx = C.dtype.is_complex
    t2 = 'C' if cplx else 'T'
    m = mask if mask is not None else ((1 if _ch(uplo) == 'L' else 2), 1 << 40, 1, 0, 1, 0, 0, 0, 0)
    if _ch(trans) == 'N':
        return gemm(alpha, A, A, beta, C, 'N', t2, m)
    return gemm(alpha, A, A, beta, C, t2, 'N', m)


def syrk(uplo, trans, alpha, A, beta, C, mask=None):
    m = mask if mask is not None else ((1 if _ch(uplo) == 'L' else 2), 1 << 40, 1, 0, 1, 0, 0, 0, 0)
    if _ch(trans) == 'N':
        return gemm(alpha, A, A, beta, C, 'N', 'T', m)
    return gemm(alpha, A, A, beta, C, 'T', 'N', m)


def her2k(uplo, trans, alpha, A, B, beta, C, mask=None):
    cplx = C.dtype.is_complex
    t2 = 'C' if cplx else 'T'
    m = mask if mask is not None else ((1 if _ch(uplo) == 'L' else 2), 1 << 40, 1, 0, 1, 0, 0, 0, 0)
    a2 = complex(alpha).conjugate() if cplx else alpha
    if _ch(trans) == 'N':
        gemm(alpha, A, B, beta, C, 'N', t2, m)
        return gemm(a2, B, A, 1.0, C, 'N', t2, m)
    gemm(alpha, A, B, beta, C, t2, 'N', m)
    return gemm(a2, B, A, 1.0, C, t2, 'N', m)


def syr2k(uplo, trans, alpha, A, B, beta, C, mask=None):
    m = mask if mask is not None else ((1 if _ch(uplo) == 'L' else 2), 1 << 40, 1, 0, 1, 0, 0, 0, 0)
    if _ch(trans) == 'N':
        gemm(alpha, A, B, beta, C, 'N', 'T', m)
        return gemm(alpha, B, A, 1.0, C, 'N', 'T', m)
    gemm(alpha, A, B, beta, C, 'T', 'N', m)
    return gemm(alpha, B, A, 1.0, C, 'T', 'N', m)


def trsm(side, uplo, trans, diag, alpha, A, B):
    """op(A) X = alpha B (Left) or X op(A) = alpha B (Right); B <- X."""
    _chk(A); _chk(B, "B")
    m, n = B.shape
    if m == 0 or n == 0:
        return B
    if _FLOPS is not None:
        _FLOPS[0] += (m * m * n) if _ch(side) == 'L' else (m * n * n)
    kmod(B).trsm(code(B.dtype), _ch(side), _ch(uplo), _ch(trans), _ch(diag), m, n, _c(alpha),
                 A.data_ptr(), ld(A), B.data_ptr(), ld(B), stream(B))
    return B


def trmm(side, uplo, trans, diag, alpha, A, B):
    _chk(A); _chk(B, "B")
    m, n = B.shape
    if m == 0 or n == 0:
        return B
    if _FLOPS is not None:
        _FLOPS[0] += (m * m * n) if _ch(side) == 'L' else (m * n * n)
    kmod(B).trmm(code(B.dtype), _ch(side), _ch(uplo), _ch(trans), _ch(diag), m, n, _c(alpha),
                 A.data_ptr(), ld(A), B.data_ptr(), ld(B), stream(B))
    return B


# ------------------------------------------------------------- factorizations
def info_tensor(like: torch.Tensor, n=1):
    return torch.zeros(n, dtype=torch.int64, device=like.device)


def potrf(uplo, A, info=None):
    """Tile Cholesky in place; info (int64 tensor on A's device) gets 0 or the
    1-based failing column.  No host sync."""
    _chk(A)
    n = A.shape[0]
    if info is None:
        info = info_tensor(A)
    kmod(A).potrf(code(A.dtype), _ch(uplo), n, A.data_ptr(), ld(A), info.data_ptr(), stream(A))
    return info


def _work(dev):
    key = str(dev)
    w = _WORK.get(key)
    if w is None:
        nbytes = max(64, int(kmod(torch.empty(0, device=dev)).getrf_work_bytes()))
        w = torch.zeros(nbytes // 8 + 8, dtype=torch.int64, device=dev)
        _WORK[key] = w
    return w


def getrf(A, ipiv, info=None, threshold=1.0, nopiv=False):
    """LU panel with partial pivoting: ipiv (int64, length min(m,n)) gets
    0-based pivot rows relative to A's first row."""
    _chk(A)
    m, n = A.shape
    if info is None:
        info = info_tensor(A)
    w = _work(A.device) if A.is_cuda else None
    kmod(A).getrf(code(A.dtype), m, n, A.data_ptr(), ld(A), ipiv.data_ptr() if ipiv is not None else 0,
                  info.data_ptr(), float(threshold), bool(nopiv), w.data_ptr() if w is not None else 0, stream(A))
    return info


def laswp(A, ipiv, k1, k2, ioff=0, incx=1):
    """Apply row interchanges ipiv[k1:k2] (rows ipiv[k]-ioff <-> k) to A."""
    _chk(A)
    if A.shape[1] == 0 or k2 <= k1:
        return A
    kmod(A).laswp(code(A.dtype), A.shape[1], A.data_ptr(), ld(A), k1, k2, ipiv.data_ptr(), ioff, incx, stream(A))
    return A


def laswp_cols(A, ipiv, k1, k2, ioff=0, incx=1):
    """Apply column interchanges ipiv[k1:k2] (cols ipiv[k]-ioff <-> k) to A:
    the row interchanges of A^T, with whole-cache-line accesses."""
    _chk(A)
    if A.shape[0] == 0 or k2 <= k1:
        return A
    kmod(A).laswp_cols(code(A.dtype), A.shape[0], A.data_ptr(), ld(A), k1, k2, ipiv.data_ptr(), ioff, incx,
                       stream(A))
    return A


def laswp_cols_plan(A, plan):
    """laswp_cols with a plan from swap_plan (folded once per panel)."""
    _chk(A)
    if A.shape[0] and A.shape[1]:
        kmod(A).laswp_cols_plan(code(A.dtype), A.shape[0], A.data_ptr(), ld(A), plan.data_ptr(), stream(A))
    return A


def spin_ns(ns, like):
    """Hold the current stream of ``like``'s device for ``ns`` nanoseconds
    (one-wave wall-clock spin; the loopback transport's link model)."""
    if like.is_cuda and ns > 0:
        kmod(like).spin_ns(float(ns), stream(like))


def cols_move(A, B, idx, scatter=False):
    """B[:, j] = A[:, idx[j]] (gather) or B[:, idx[j]] = A[:, j] (scatter):
    one launch of the device column-copy kernel, elements of 8 or 16 bytes
    moved as doubles (callers with other element sizes or CPU tensors use
    torch's index ops)."""
    _chk(A); _chk(B, "B")
    k = A.element_size() // 8
    nc = (B if not scatter else A).shape[1]
    if A.shape[0] == 0 or nc == 0:
        return B
    _native.hip().cols_copy(A.shape[0] * k, nc, A.data_ptr(), ld(A) * k, idx.data_ptr(), B.data_ptr(), ld(B) * k,
                            1 if scatter else 0, stream(B))
    return B


def row_gather(A, B, perm):
    """B[i, :] = A[perm[i], :]."""
    m, n = B.shape
    if m == 0 or n == 0:
        return B
    kmod(B).row_gather(code(B.dtype), m, n, A.data_ptr(), ld(A), B.data_ptr(), ld(B), perm.data_ptr(), stream(B))
    return B


def row_scatter(A, B, perm):
    """B[perm[i], :] = A[i, :]."""
    m, n = A.shape
    if m == 0 or n == 0:
        return B
    kmod(B).row_scatter(code(B.dtype), m, n, A.data_ptr(), ld(A), B.data_ptr(), ld(B), perm.data_ptr(), stream(B))
    return B


# ------------------------------------------- distributed row interchange
def swap_plan(ipiv, k1, k2, ioff=0, out=None, incx=1):
    """Fold the swap sequence ipiv[k1:k2) (values - ioff are absolute rows)
    into a plan of touched rows (SwapPlan layout, stays on ipiv's device)."""
    mod = kmod(ipiv)
    if out is None:
        out = torch.empty(int(mod.swap_plan_bytes()) // 8 + 1, dtype=torch.int64, device=ipiv.device)
    mod.swap_plan(int(k1), int(k2), ipiv.data_ptr(), int(ioff), int(incx), out.data_ptr(), stream(ipiv))
    return out


def xchg_gather(plan, A, X, nb, p, pr):
    """X[t, :] = A[local(src_t), :] for the plan's touched rows owned by
    process row pr (block-cyclic rows, tile nb), 0 elsewhere; X has 2kb rows."""
    _chk(A); _chk(X, "X")
    S, n = X.shape
    if S and n:
        kmod(X).xchg_gather(code(X.dtype), plan.data_ptr(), S, n, A.data_ptr(), ld(A), X.data_ptr(), ld(X),
                            int(nb), int(p), int(pr), stream(X))
    return X


def xchg_scatter(plan, X, A, nb, p, pr):
    """A[local(dst_t), :] = X[t, :] for the touched rows owned by pr."""
    _chk(A); _chk(X, "X")
    S, n = X.shape
    if S and n:
        kmod(A).xchg_scatter(code(A.dtype), plan.data_ptr(), S, n, X.data_ptr(), ld(X), A.data_ptr(), ld(A),
                             int(nb), int(p), int(pr), stream(A))
    return A


def sel_to_ipiv(sel, r0, ipiv):
    """Pivot SET sel (global rows, in order) -> LAPACK swap sequence ipiv
    (relative to r0), as tournament pivoting needs."""
    kb = sel.shape[0]
    if kb:
        kmod(sel).sel_to_ipiv(sel.data_ptr(), kb, int(r0), ipiv.data_ptr(), stream(sel))
    return ipiv


def tri_inv(uplo, diag, A, W=None):
    """W = inverse of the uplo triangle of A (diag 'U': unit, A's diagonal
    not read); A untouched.  W: n x n column-major (allocated if None), its
    other triangle zero."""
    _chk(A)
    n = A.shape[0]
    if W is None:
        W = colmajor_empty(n, n, A.dtype, A.device)
    if n:
        kmod(A).tri_inv(code(A.dtype), _ch(uplo), _ch(diag), n, A.data_ptr(), ld(A), W.data_ptr(), ld(W), stream(A))
    return W


def trtri(uplo, diag, A, info=None):
    _chk(A)
    if info is None:
        info = info_tensor(A)
    kmod(A).trtri(code(A.dtype), _ch(uplo), _ch(diag), A.shape[0], A.data_ptr(), ld(A), info.data_ptr(), stream(A))
    return info


def _qr_work(dev):
    key = "qr:" + str(dev)
    w = _WORK.get(key)
    if w is None:
        nbytes = max(64, int(kmod(torch.empty(0, device=dev)).geqrf_work_bytes()))
        w = torch.zeros(nbytes // 8 + 8, dtype=torch.int64, device=dev)
        _WORK[key] = w
    return w


def geqrf(A, tau, T=None, V=None):
    """Householder QR of a panel A (m x n) in place: R on/above the diagonal,
    the reflectors below it, tau[min(m,n)].  Optionally also returns the
    compact-WY factor T (k x k upper, I - V T V^H = H_0 ... H_{k-1}) and the
    explicit unit-lower V (m x k).  Device: recursive MFMA panel
    (csrc/hip/geqrf.hip); host: native Householder + larft."""
    _chk(A)
    m, n = A.shape
    k = min(m, n)
    if T is None:
        T = colmajor_empty(k, k, A.dtype, A.device)
    if V is None:
        V = colmajor_empty(m, k, A.dtype, A.device)
    if m == 0 or n == 0:
        return T, V
    if A.is_cuda:
        w = _qr_work(A.device)
        kmod(A).geqrf(code(A.dtype), m, n, A.data_ptr(), ld(A), tau.data_ptr(), T.data_ptr(), ld(T),
                      V.data_ptr(), ld(V), w.data_ptr(), stream(A))
    else:
        _native._host.geqrf(code(A.dtype), m, n, A.data_ptr(), ld(A), tau.data_ptr())
        v_explicit(A[:, :k], V)
        T.zero_()
        larft(V, tau[:k], T)
    return T, V


def tpqrt(l, A, B, T=None, V=None, tau=None, ib=32):
    """Triangle-pentagonal QR (tile::tpqrt, src/internal/Tile_tpqrt.hh:142):
    QR of [A; B] with A n x n upper triangular and B m x n pentagonal (the
    last ``l`` rows upper trapezoidal, l = 0: B full, l = min(m, n): B
    triangular).  R overwrites A's upper triangle, the reflectors' B parts
    overwrite B's pentagon; Q = I - [I; V] T [I; V]^H.  Returns (T, V, tau)
    with T the full n x n compact-WY factor and V the explicit m x n
    reflector block (zeros outside the pentagon).

    Blocked: each ib-column panel by one workgroup (csrc/hip/tpqrt.hip),
    the tile's trailing columns by the block reflector as MFMA GEMM/TRMM
    (tprfb), and the panel T's merged into the full T by
    T12 = -T11 (V1^H V2) T22 (the unit top parts of the reflectors are
    disjoint, so only V_B enters)."""
    _chk(A); _chk(B, "B")
    m, n = B.shape
    if A.shape[0] < n or A.shape[1] != n:
        raise SlateError("tpqrt: A must be n x n with n = B.shape[1]")
    if not 0 <= l <= min(m, n) and not (l == m == 0):
        raise SlateError("tpqrt: need 0 <= l <= min(m, n)")
    dt, dev = B.dtype, B.device
    if T is None:
        T = colmajor_zeros(n, n, dt, dev)
    if V is None:
        V = colmajor_zeros(m, n, dt, dev)
    if tau is None:
        tau = torch.zeros(n, dtype=dt, device=dev)
    if n == 0:
        return T, V, tau
    if m == 0:
        tau.zero_()
        T.zero_()
        return T, V, tau
    ib = max(1, min(int(ib), 64))
    mod = kmod(B)
    ct = 'C' if dt.is_complex else 'T'
    for j0 in range(0, n, ib):
        jb = min(ib, n - j0)
        mod.tpqrt_panel(code(dt), m, int(l), j0, jb, A[j0:, j0:].data_ptr(), ld(A), B[:, j0:].data_ptr(), ld(B),
                        V[:, j0:].data_ptr(), ld(V), tau[j0:].data_ptr(), T[j0:, j0:].data_ptr(), ld(T), stream(B))
        if j0 + jb < n:
            tpmqrt('L', 'C', V[:, j0:j0 + jb], T[j0:j0 + jb, j0:j0 + jb], A[j0:j0 + jb, j0 + jb:], B[:, j0 + jb:])
        if j0:
            G = T[:j0, j0:j0 + jb]
            gemm(1.0, V[:, :j0], V[:, j0:j0 + jb], 0.0, G, transA=ct)
            trmm('L', 'U', 'N', 'N', 1.0, T[:j0, :j0], G)
            trmm('R', 'U', 'N', 'N', -1.0, T[j0:j0 + jb, j0:j0 + jb], G)
    return T, V, tau


def tpmqrt(side, trans, V, T, A, B):
    """Apply Q (trans 'N') or Q^H ('C'/'T') of a tpqrt factorization,
    Q = I - [I; V] T [I; V]^H, to the stacked pair (tile::tpmqrt,
    src/internal/Tile_tpmqrt.hh:99): side 'L' acts on [A; B] (A k x nc,
    B m x nc), side 'R' on [A B] (A nr x k, B nr x m).  Three MFMA
    GEMM-class launches plus a copy: W = A + V^H B (or A + B V),
    W = op(T) W (or W op(T)), A -= W, B -= V W (or W V^H)."""
    _chk(A); _chk(B, "B"); _chk(V, "V")
    dt = B.dtype
    ct = 'C' if dt.is_complex else 'T'
    conj = _ch(trans) != 'N'
    k = T.shape[0]
    if k == 0:
        return A, B
    if _ch(side) == 'L':
        nc = A.shape[1]
        if nc == 0:
            return A, B
        W = colmajor_empty(k, nc, dt, A.device)
        W.copy_(A)
        gemm(1.0, V, B, 1.0, W, transA=ct)
        trmm('L', 'U', ct if conj else 'N', 'N', 1.0, T, W)
        geadd(-1.0, W, 1.0, A)
        gemm(-1.0, V, W, 1.0, B)
    else:
        nr = A.shape[0]
        if nr == 0:
            return A, B
        W = colmajor_empty(nr, k, dt, A.device)
        W.copy_(A)
        gemm(1.0, B, V, 1.0, W)
        trmm('R', 'U', ct if conj else 'N', 'N', 1.0, T, W)
        geadd(-1.0, W, 1.0, A)
        gemm(-1.0, W, V, 1.0, B, transB=ct)
    return A, B


def tplqt(l, A, B, ib=32):
    """Triangle-pentagonal LQ (tile::tplqt, src/internal/Tile_tplqt.hh:145):
    LQ of [A B] with A k x k lower triangular and B k x m pentagonal (the
    last ``l`` columns lower trapezoidal).  Computed as the tpqrt of the
    conjugate transposes; L overwrites A's lower triangle, the reflectors'
    B parts overwrite B.  Returns (T, W, tau): Q = I - [I W] T^H [I W]^H
    acting on the right, W = V^H (k x m)."""
    Ah = as_colmajor(A.mH.contiguous())
    Bh = as_colmajor(B.mH.contiguous())
    T, V, tau = tpqrt(l, Ah, Bh, ib=ib)
    A.copy_(Ah.mH)
    B.copy_(Bh.mH)
    return T, as_colmajor(V.mH.contiguous()), tau


def tpmlqt(side, trans, W, T, A, B):
    """Apply Q or Q^H of a tplqt factorization (tile::tpmlqt,
    src/internal/Tile_tpmlqt.hh:99).  The LQ factor of [A B] is the
    conjugate transpose of the QR factor of [A; B]^H, so Q_lq = Q_qr^H with
    V = W^H: this is tpmqrt with the transposition flipped."""
    V = as_colmajor(W.mH.contiguous())
    return tpmqrt(side, 'N' if _ch(trans) != 'N' else 'C', V, T, A, B)


def v_explicit(A, V):
    """V = unit-lower-trapezoidal part of A (reflectors), zeros above."""
    m, k = V.shape
    if m == 0 or k == 0:
        return V
    if A.is_cuda:
        kmod(A).v_explicit(code(A.dtype), m, k, A.data_ptr(), ld(A), V.data_ptr(), ld(V), stream(A))
    else:
        V.copy_(torch.tril(A[:m, :k], -1))
        V.diagonal().fill_(1)
    return V


def gelqf(A, tau):
    """Householder LQ of a panel in place (L on/below the diagonal, the
    reflectors' conjugates to the right, LAPACK layout).  Host: native
    kernel; device: the GPU QR of A^H written back as its conjugate
    transpose (gelqf(A) is geqrf(A^H)^H)."""
    _chk(A)
    if A.is_cuda:
        Ah = as_colmajor(A.mH.contiguous())
        geqrf(Ah, tau)
        A.copy_(Ah.mH)
        return tau
    _native._host.gelqf(code(A.dtype), A.shape[0], A.shape[1], A.data_ptr(), ld(A), tau.data_ptr())
    return tau


def larft(V, tau, T):
    """Compact-WY T of the reflectors V (host tensors; the device QR panels
    return T themselves)."""
    if V.is_cuda:
        raise SlateError("larft: host tensors only (device panels produce T in ops.geqrf)")
    _native._host.larft(code(V.dtype), V.shape[0], tau.shape[0], V.data_ptr(), ld(V), tau.data_ptr(),
                        T.data_ptr(), ld(T))
    return T


# --------------------------------------------------------------------- aux
def geset(offdiag, diag, A, uplo='G'):
    _chk(A)
    m, n = A.shape
    if m and n:
        kmod(A).geset(code(A.dtype), _ch(uplo), m, n, _c(offdiag), _c(diag), A.data_ptr(), ld(A), stream(A))
    return A


def gescale(alpha, A, uplo='G'):
    _chk(A)
    m, n = A.shape
    if m and n:
        kmod(A).gescale(code(A.dtype), _ch(uplo), m, n, _c(alpha), A.data_ptr(), ld(A), stream(A))
    return A


def geadd(alpha, A, beta, B, uplo='G'):
    """B = alpha A + beta B."""
    _chk(A); _chk(B, "B")
    m, n = B.shape
    if m and n:
        kmod(B).geadd(code(B.dtype), _ch(uplo), m, n, _c(alpha), A.data_ptr(), ld(A), _c(beta),
                      B.data_ptr(), ld(B), stream(B))
    return B


def gecopy(A, B, uplo='G', trans='N'):
    """B = op(A) with precision conversion (B is m x n)."""
    _chk(A); _chk(B, "B")
    m, n = B.shape
    if m and n:
        kmod(B).gecopy(code(A.dtype), code(B.dtype), _ch(uplo), _ch(trans), m, n, A.data_ptr(), ld(A),
                       B.data_ptr(), ld(B), stream(B))
    return B


def gecopy_mask(A, B, mask, real_diag=False):
    """B = A where the block-cyclic triangle ``mask`` (the GEMM TriMask tuple
    (mode, nb, p, pr, q, pc, row_off, col_off, diag_off)) keeps the element,
    0 elsewhere; ``real_diag`` drops the imaginary part of kept diagonal
    elements (Hermitian).  One kernel launch."""
    _chk(A); _chk(B, "B")
    m, n = B.shape
    if m and n:
        kmod(B).gecopy_mask(code(B.dtype), tuple(int(x) for x in mask), m, n, A.data_ptr(), ld(A),
                            B.data_ptr(), ld(B), 1 if real_diag else 0, stream(B))
    return B


def gescale_row_col(equed, r, c, A):
    m, n = A.shape
    if m and n:
        kmod(A).gescale_row_col(code(A.dtype), _ch(equed), m, n, r.data_ptr() if r is not None else 0,
                                c.data_ptr() if c is not None else 0, A.data_ptr(), ld(A), stream(A))
    return A


def butterfly(A, diag, depth, trans=False, side='L'):
    """Random butterfly transform in place: side 'L' A := op(W) A (rows),
    side 'R' A := A op(W)^T (op(W) applied to the column index), op(W) = W^T
    when ``trans``; W = W_depth ... W_1, diag (depth x n real, row l = level
    l's butterfly diagonals, n = length of the transformed dimension).  One
    pass over A for all levels."""
    _chk(A)
    m, n = A.shape
    rows = side.upper() == 'L'
    nidx, nother = (m, n) if rows else (n, m)
    if nidx and nother:
        kmod(A).butterfly(code(A.dtype), bool(trans), rows, int(depth), nidx, nother, A.data_ptr(), ld(A),
                          diag.data_ptr(), diag.stride(0), stream(A))
    return A


def genorm_local(norm, A, uplo='G', diag='N', herm=0):
    """Local norm contributions: returns (colvals, rowvals) real tensors on
    A's device: 'M'/'1' -> per-column max/sum, 'F' -> per-column
    (scale, sumsq) pairs (n x 2), 'I' -> per-row sums; symmetric/Hermitian
    storage adds the mirrored contributions to rowvals (herm 1: symmetric,
    2: Hermitian -- the diagonal's real part only, as LAPACK lanhe)."""
    _chk(A)
    m, n = A.shape
    rdt = _native.REAL_OF[A.dtype]
    nc = 2 * n if _ch(norm) == 'F' else n
    out = torch.zeros(nc + m, dtype=rdt, device=A.device)
    if m and n:
        kmod(A).genorm(code(A.dtype), _ch(norm), _ch(uplo), _ch(diag), int(herm), m, n, A.data_ptr(), ld(A),
                       out.data_ptr(), stream(A))
    col = out[:nc].view(n, 2) if _ch(norm) == 'F' else out[:nc]
    return col, out[nc:]


def matgen(kind: int, seed: int, A, m, n, mb, p, pr, nb, q, pc, row0=0, col0=0, scale=1.0):
    _chk(A)
    mloc, nloc = A.shape
    if mloc and nloc:
        kmod(A).matgen(code(A.dtype), int(kind), int(seed) & ((1 << 64) - 1), mloc, nloc, A.data_ptr(), ld(A),
                       m, n, mb, p, pr, nb, q, pc, row0, col0, float(scale), *( [stream(A)] if A.is_cuda else []))
    return A


# ------------------------------------------------------------- eig / svd
def apply_refl(Z, V, tau, row, length, first, count, conj_tau=False):
    """Z := H_k Z for the recorded bulge-chasing reflectors k in
    [first, first+count) (disjoint row ranges: one launch).  V is
    (count_total x b) row-major, row/length int64."""
    _chk(Z, "Z")
    if count <= 0 or Z.shape[1] == 0:
        return Z
    kmod(Z).apply_refl(code(Z.dtype), Z.shape[1], Z.data_ptr(), ld(Z), V.data_ptr(), V.shape[1], tau.data_ptr(),
                       row.data_ptr(), length.data_ptr(), int(first), int(count), bool(conj_tau), stream(Z))
    return Z
