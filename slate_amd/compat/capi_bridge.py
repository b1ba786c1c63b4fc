"""Python side of the C ABI (csrc/capi/capi.cpp): raw pointers from C are
wrapped zero-copy as numpy arrays and passed to compat.lapack."""
from __future__ import annotations

import ctypes

import numpy as np

from . import lapack

_CT = {'s': (ctypes.c_float, np.float32, 1), 'd': (ctypes.c_double, np.float64, 1),
       'c': (ctypes.c_float, np.complex64, 2), 'z': (ctypes.c_double, np.complex128, 2)}


def _arr(pfx, ptr, rows, cols, ld):
    """Flat column-major array of ld*(cols-1)+rows elements at address ptr."""
    if ptr == 0 or rows <= 0 or cols <= 0:
        return np.zeros(0, dtype=_CT[pfx][1])
    ct, npdt, w = _CT[pfx]
    n = ld * (cols - 1) + rows
    raw = np.ctypeslib.as_array((ct * (n * w)).from_address(ptr))
    return raw.view(npdt)


def _iarr(ptr, n):
    return np.ctypeslib.as_array((ctypes.c_int64 * n).from_address(ptr)) if n > 0 else np.zeros(0, np.int64)


def call(name, *args):
    pfx, rt = name[0], name[1:]
    f = getattr(lapack, name)
    if rt == "gemm":
        ta, tb, m, n, k, al, a, lda, b, ldb, be, c, ldc = args
        ar, ac = (m, k) if ta.upper() == 'N' else (k, m)
        br, bc = (k, n) if tb.upper() == 'N' else (n, k)
        return f(ta, tb, m, n, k, al, _arr(pfx, a, ar, ac, lda), lda, _arr(pfx, b, br, bc, ldb), ldb, be,
                 _arr(pfx, c, m, n, ldc), ldc)
    if rt in ("potrf", "potri"):
        uplo, n, a, lda = args
        return f(uplo, n, _arr(pfx, a, n, n, lda), lda)
    if rt in ("potrs", "posv"):
        uplo, n, nrhs, a, lda, b, ldb = args
        return f(uplo, n, nrhs, _arr(pfx, a, n, n, lda), lda, _arr(pfx, b, n, nrhs, ldb), ldb)
    if rt == "getrf":
        m, n, a, lda, ip = args
        return f(m, n, _arr(pfx, a, m, n, lda), lda, _iarr(ip, min(m, n)))
    if rt == "getrs":
        t, n, nrhs, a, lda, ip, b, ldb = args
        return f(t, n, nrhs, _arr(pfx, a, n, n, lda), lda, _iarr(ip, n), _arr(pfx, b, n, nrhs, ldb), ldb)
    if rt == "gesv":
        n, nrhs, a, lda, ip, b, ldb = args
        return f(n, nrhs, _arr(pfx, a, n, n, lda), lda, _iarr(ip, n), _arr(pfx, b, n, nrhs, ldb), ldb)
    if rt == "trsm":
        side, uplo, ta, diag, m, n, al, a, lda, b, ldb = args
        k = m if side.upper() == 'L' else n
        return f(side, uplo, ta, diag, m, n, al, _arr(pfx, a, k, k, lda), lda, _arr(pfx, b, m, n, ldb), ldb)
    if rt == "gels":
        t, m, n, nrhs, a, lda, b, ldb = args
        return f(t, m, n, nrhs, _arr(pfx, a, m, n, lda), lda, _arr(pfx, b, max(m, n), nrhs, ldb), ldb)
    if rt in ("syev", "heev"):
        jobz, uplo, n, a, lda, w = args
        wv = np.ctypeslib.as_array((_CT[pfx][0] * n).from_address(w))
        return f(jobz, uplo, n, _arr(pfx, a, n, n, lda), lda, wv)
    if rt == "gesvd":
        ju, jv, m, n, a, lda, s, u, ldu, vt, ldvt = args
        k = min(m, n)
        sv = np.ctypeslib.as_array((_CT[pfx][0] * k).from_address(s))
        return f(ju, jv, m, n, _arr(pfx, a, m, n, lda), lda, sv, _arr(pfx, u, m, k, ldu) if u else None, ldu,
                 _arr(pfx, vt, k, n, ldvt) if vt else None, ldvt)
    if rt == "lange":
        nrm, m, n, a, lda = args
        return f(nrm, m, n, _arr(pfx, a, m, n, lda), lda)
    raise ValueError(name)
