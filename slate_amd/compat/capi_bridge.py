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
    return _call_more(pfx, rt, f, *args)


_RT = {'s': 's', 'd': 'd', 'c': 's', 'z': 'd'}       # real type of each prefix


def _scalar(pfx, re, im=0.0):
    return complex(re, im) if pfx in "cz" else re


def _out(pfx, ptr, v):
    """Write one real (s/d -> float/double) or int64 ('i') output value."""
    ct = {'s': ctypes.c_float, 'd': ctypes.c_double, 'i': ctypes.c_int64, 'i32': ctypes.c_int32}[pfx]
    if ptr:
        ct.from_address(ptr).value = v


def _call_more(pfx, rt, f, *args):
    """LAPACK-style routines added in round 3 (lapack_api/lapack_trmm.cc,
    _syrk, _syr2k, _symm, _hemm, _herk, _her2k, _getri, _gesv_mixed, _lansy,
    _lanhe, _lantr, _gecon, _pocon, _trcon, _heevd).  Complex scalars arrive
    as (re, im) pairs; condition numbers / iteration counts are written to
    the caller's output pointers."""
    if rt == "trmm":
        side, uplo, ta, diag, m, n, al, a, lda, b, ldb = args
        k = m if side.upper() == 'L' else n
        return f(side, uplo, ta, diag, m, n, al, _arr(pfx, a, k, k, lda), lda,
                 _arr(pfx, b, m, n, ldb), ldb)
    if rt in ("syrk", "herk"):
        uplo, tr, n, k, al, a, lda, be, c, ldc = args
        ar, ac = (n, k) if tr.upper() == 'N' else (k, n)
        return f(uplo, tr, n, k, al, _arr(pfx, a, ar, ac, lda), lda, be, _arr(pfx, c, n, n, ldc), ldc)
    if rt in ("syr2k", "her2k"):
        uplo, tr, n, k, are, aim, a, lda, b, ldb, be, c, ldc = args
        ar, ac = (n, k) if tr.upper() == 'N' else (k, n)
        return f(uplo, tr, n, k, _scalar(pfx, are, aim), _arr(pfx, a, ar, ac, lda), lda,
                 _arr(pfx, b, ar, ac, ldb), ldb, be, _arr(pfx, c, n, n, ldc), ldc)
    if rt in ("symm", "hemm"):
        side, uplo, m, n, are, aim, a, lda, b, ldb, bre, bim, c, ldc = args
        k = m if side.upper() == 'L' else n
        return f(side, uplo, m, n, _scalar(pfx, are, aim), _arr(pfx, a, k, k, lda), lda,
                 _arr(pfx, b, m, n, ldb), ldb, _scalar(pfx, bre, bim), _arr(pfx, c, m, n, ldc), ldc)
    if rt == "getri":
        n, a, lda, ip = args
        return f(n, _arr(pfx, a, n, n, lda), lda, _iarr(ip, n))
    if rt == "gesv_mixed":
        n, nrhs, a, lda, ip, b, ldb, x, ldx, it = args
        info, iters = f(n, nrhs, _arr(pfx, a, n, n, lda), lda, _iarr(ip, n), _arr(pfx, b, n, nrhs, ldb), ldb,
                        _arr(pfx, x, n, nrhs, ldx), ldx)
        _out('i', it, int(iters))
        return info
    if rt in ("lansy", "lanhe"):
        nrm, uplo, n, a, lda = args
        return f(nrm, uplo, n, _arr(pfx, a, n, n, lda), lda)
    if rt == "lantr":
        nrm, uplo, diag, m, n, a, lda = args
        return f(nrm, uplo, diag, m, n, _arr(pfx, a, m, n, lda), lda)
    if rt == "gecon":
        nrm, n, a, lda, anorm, rc = args
        info, r = f(nrm, n, _arr(pfx, a, n, n, lda), lda, anorm)
        _out(_RT[pfx], rc, r)
        return info
    if rt == "pocon":
        uplo, n, a, lda, anorm, rc = args
        info, r = f(uplo, n, _arr(pfx, a, n, n, lda), lda, anorm)
        _out(_RT[pfx], rc, r)
        return info
    if rt == "trcon":
        nrm, uplo, diag, n, a, lda, rc = args
        info, r = f(nrm, uplo, diag, n, _arr(pfx, a, n, n, lda), lda)
        _out(_RT[pfx], rc, r)
        return info
    if rt in ("syevd", "heevd"):
        jobz, uplo, n, a, lda, w = args
        wv = np.ctypeslib.as_array((_CT[_RT[pfx]][0] * n).from_address(w))
        return f(jobz, uplo, n, _arr(pfx, a, n, n, lda), lda, wv)
    raise ValueError(pfx + rt)


# ---------------------------------------------------------------- ScaLAPACK
# pd*_ symbols of libslate_amd_c.so: descriptors arrive as 9 ints, local
# arrays as raw pointers sized from the descriptor (lld x local columns).
def _desc_arr(pfx, ptr, desc):
    from . import scalapack as S
    ctxt, n, nb, csrc, lld = desc[1], desc[3], desc[5], desc[7], desc[8]
    _, q, _, pc = S.blacs_gridinfo(ctxt)
    nloc = S.numroc(n, nb, pc, csrc, q)
    return _arr(pfx, ptr, max(lld, 1), nloc, max(lld, 1)) if nloc else np.zeros(0, dtype=_CT[pfx][1])


def _local_rows(desc):
    """(global row of each local row) of this rank for descriptor desc."""
    from . import scalapack as S
    ctxt, m, mb, rsrc = desc[1], desc[2], desc[4], desc[6]
    p, _, pr, _ = S.blacs_gridinfo(ctxt)
    mloc = S.numroc(m, mb, pr, rsrc, p)
    lr = np.arange(mloc, dtype=np.int64)
    return ((lr // mb) * p + pr) * mb + lr % mb


def _ipiv_to_local(piv, ia, desc, ip):
    """ScaLAPACK ipiv is distributed like the rows of A: local row i holds
    the (1-based, global) pivot row of global row l2g(i).  piv: pivots of
    the sub-matrix at ia, 1-based relative to it."""
    g = _local_rows(desc)
    out = np.ctypeslib.as_array((ctypes.c_int32 * max(len(g), 1)).from_address(ip))
    off = int(ia) - 1
    for i, gr in enumerate(g):
        k = gr - off
        if 0 <= k < len(piv):
            out[i] = off + int(piv[k])


def _ipiv_from_local(ip, ia, n, desc):
    """Rebuild the sub-matrix pivot vector (1-based, relative to ia) from the
    distributed ipiv: every rank contributes its rows, one max-reduction."""
    import torch
    from ..parallel import comm as C
    g = _local_rows(desc)
    loc = np.ctypeslib.as_array((ctypes.c_int32 * max(len(g), 1)).from_address(ip))
    off = int(ia) - 1
    full = torch.zeros(n, dtype=torch.int64)
    for i, gr in enumerate(g):
        k = gr - off
        if 0 <= k < n:
            full[k] = int(loc[i]) - off
    w = C.world()
    if w.size > 1:
        w.allreduce(full, "max")
    return full.numpy()


def scalapack_call(name, *args):
    """ScaLAPACK entry points by name ('pdpotrf', ...): args are plain values,
    pointers and 9-int descriptors (as tuples)."""
    from . import scalapack as S
    pfx, rt = name[1], name[2:]
    f = getattr(S, name)
    if rt == "gemm":
        ta, tb, m, n, k, al, a, ia, ja, da, b, ib, jb, db, be, c, ic, jc, dc = args
        return f(ta, tb, m, n, k, al, _desc_arr(pfx, a, da), ia, ja, da, _desc_arr(pfx, b, db), ib, jb, db, be,
                 _desc_arr(pfx, c, dc), ic, jc, dc)
    if rt == "potrf":
        uplo, n, a, ia, ja, da = args
        return f(uplo, n, _desc_arr(pfx, a, da), ia, ja, da)
    if rt in ("potrs", "posv"):
        uplo, n, nrhs, a, ia, ja, da, b, ib, jb, db = args
        return f(uplo, n, nrhs, _desc_arr(pfx, a, da), ia, ja, da, _desc_arr(pfx, b, db), ib, jb, db)
    if rt == "getrf":
        m, n, a, ia, ja, da, ip = args
        piv = np.zeros(min(m, n), dtype=np.int64)
        info = f(m, n, _desc_arr(pfx, a, da), ia, ja, da, piv)
        _ipiv_to_local(piv, ia, da, ip)
        return info
    if rt in ("getrs", "gesv"):
        if rt == "getrs":
            t, n, nrhs, a, ia, ja, da, ip, b, ib, jb, db = args
            piv = _ipiv_from_local(ip, ia, n, da)
            return f(t, n, nrhs, _desc_arr(pfx, a, da), ia, ja, da, piv, _desc_arr(pfx, b, db), ib, jb, db)
        n, nrhs, a, ia, ja, da, ip, b, ib, jb, db = args
        piv = np.zeros(n, dtype=np.int64)
        info = f(n, nrhs, _desc_arr(pfx, a, da), ia, ja, da, piv, _desc_arr(pfx, b, db), ib, jb, db)
        _ipiv_to_local(piv, ia, da, ip)
        return info
    if rt == "trsm":
        side, uplo, ta, diag, m, n, al, a, ia, ja, da, b, ib, jb, db = args
        return f(side, uplo, ta, diag, m, n, al, _desc_arr(pfx, a, da), ia, ja, da, _desc_arr(pfx, b, db), ib, jb,
                 db)
    if rt == "lange":
        nrm, m, n, a, ia, ja, da = args
        return f(nrm, m, n, _desc_arr(pfx, a, da), ia, ja, da)
    return _scalapack_more(pfx, rt, f, *args)


def _rvec(pfx, ptr, n):
    """Replicated real vector (eigen / singular values) at ptr."""
    return np.ctypeslib.as_array((_CT[_RT[pfx]][0] * max(n, 1)).from_address(ptr))[:n]


def _scalapack_more(pfx, rt, f, *args):
    """p?xxx_ interposers added in round 3 (scalapack_api/scalapack_trmm.cc,
    _herk, _syrk, _her2k, _syr2k, _hemm, _symm, _potri, _getri, _lanhe,
    _lansy, _lantr, _gecon, _pocon, _trcon, _gesv_mixed, _heev, _heevd,
    _gesvd, _gels).  Workspace arguments of the Fortran interfaces are
    ignored (a workspace query, lwork = -1, is answered in the C layer)."""
    D = lambda ptr, d: _desc_arr(pfx, ptr, d)      # noqa: E731
    if rt == "trmm":
        side, uplo, ta, diag, m, n, al, a, ia, ja, da, b, ib, jb, db = args
        return f(side, uplo, ta, diag, m, n, al, D(a, da), ia, ja, da, D(b, db), ib, jb, db)
    if rt in ("syrk", "herk"):
        uplo, tr, n, k, al, a, ia, ja, da, be, c, ic, jc, dc = args
        return f(uplo, tr, n, k, al, D(a, da), ia, ja, da, be, D(c, dc), ic, jc, dc)
    if rt in ("syr2k", "her2k"):
        uplo, tr, n, k, are, aim, a, ia, ja, da, b, ib, jb, db, be, c, ic, jc, dc = args
        return f(uplo, tr, n, k, _scalar(pfx, are, aim), D(a, da), ia, ja, da, D(b, db), ib, jb, db, be,
                 D(c, dc), ic, jc, dc)
    if rt in ("symm", "hemm"):
        side, uplo, m, n, are, aim, a, ia, ja, da, b, ib, jb, db, bre, bim, c, ic, jc, dc = args
        return f(side, uplo, m, n, _scalar(pfx, are, aim), D(a, da), ia, ja, da, D(b, db), ib, jb, db,
                 _scalar(pfx, bre, bim), D(c, dc), ic, jc, dc)
    if rt == "potri":
        uplo, n, a, ia, ja, da = args
        return f(uplo, n, D(a, da), ia, ja, da)
    if rt == "getri":
        n, a, ia, ja, da, ip = args
        piv = _ipiv_from_local(ip, ia, n, da)
        return f(n, D(a, da), ia, ja, da, piv)
    if rt in ("lansy", "lanhe"):
        nrm, uplo, n, a, ia, ja, da = args
        return f(nrm, uplo, n, D(a, da), ia, ja, da)
    if rt == "lantr":
        nrm, uplo, diag, m, n, a, ia, ja, da = args
        return f(nrm, uplo, diag, m, n, D(a, da), ia, ja, da)
    if rt == "gecon":
        nrm, n, a, ia, ja, da, anorm, rc = args
        info, r = f(nrm, n, D(a, da), ia, ja, da, anorm)
        _out(_RT[pfx], rc, r)
        return info
    if rt == "pocon":
        uplo, n, a, ia, ja, da, anorm, rc = args
        info, r = f(uplo, n, D(a, da), ia, ja, da, anorm)
        _out(_RT[pfx], rc, r)
        return info
    if rt == "trcon":
        nrm, uplo, diag, n, a, ia, ja, da, rc = args
        info, r = f(nrm, uplo, diag, n, D(a, da), ia, ja, da)
        _out(_RT[pfx], rc, r)
        return info
    if rt == "gesv_mixed":
        n, nrhs, a, ia, ja, da, ip, b, ib, jb, db, x, ix, jx, dx, it = args
        piv = np.zeros(n, dtype=np.int64)
        info, iters = f(n, nrhs, D(a, da), ia, ja, da, piv, D(b, db), ib, jb, db, D(x, dx), ix, jx, dx)
        _ipiv_to_local(piv, ia, da, ip)
        _out('i32', it, int(iters))
        return info
    if rt in ("syev", "heev", "syevd", "heevd"):
        jobz, uplo, n, a, ia, ja, da, w, z, iz, jz, dz = args
        want = str(jobz).upper()[0] == 'V'
        return f(jobz, uplo, n, D(a, da), ia, ja, da, _rvec(pfx, w, n), D(z, dz) if want else None, iz, jz,
                 dz if want else None)
    if rt == "gesvd":
        ju, jv, m, n, a, ia, ja, da, s, u, iu, ju_, du, vt, ivt, jvt, dvt = args
        wu, wv = str(ju).upper()[0] == 'V', str(jv).upper()[0] == 'V'
        return f(ju, jv, m, n, D(a, da), ia, ja, da, _rvec(pfx, s, min(m, n)), D(u, du) if wu else None, iu, ju_,
                 du if wu else None, D(vt, dvt) if wv else None, ivt, jvt, dvt if wv else None)
    if rt == "gels":
        t, m, n, nrhs, a, ia, ja, da, b, ib, jb, db = args
        return f(t, m, n, nrhs, D(a, da), ia, ja, da, D(b, db), ib, jb, db)
    raise ValueError("p" + pfx + rt)


def _ch(x):
    """A character argument: Py_BuildValue's 'C' gives str, 'i' gives int."""
    return chr(x) if isinstance(x, int) else x


def blacs(op, *args):
    """Minimal BLACS over torch.distributed: pinfo, gridinit, gridinfo."""
    from . import scalapack as S
    from ..parallel import comm as C
    import slate_amd
    if op == "init":
        slate_amd.init()
        w = C.world()
        return w.rank * 100000 + w.size        # packed (rank, size)
    if op == "gridinit":
        order, p, q = args
        slate_amd.init()
        return S.blacs_gridinit(p, q, _ch(order))
    if op == "gridinfo":
        p, q, pr, pc = S.blacs_gridinfo(args[0])
        return ((p * 10000 + q) * 10000 + pr) * 10000 + pc
    raise ValueError(op)


# ---------------------------------------------------------------- handles
# Opaque matrix handles of the C API (SLATE's slate_Matrix_create_* family,
# src/c_api/wrappers.cc): an integer id -> the distributed matrix object.
_H = {}
_NEXT = [1]


def _tdt(pfx):
    import torch
    return {'s': torch.float32, 'd': torch.float64, 'c': torch.complex64, 'z': torch.complex128}[pfx]


def _put(obj):
    h = _NEXT[0]
    _NEXT[0] += 1
    _H[h] = obj
    return h


def handle(op, *args):
    import torch
    import slate_amd as sl
    if op == "create":
        kind, pfx, m, n, nb, p, q = args
        sl.init()
        dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
        dt = _tdt(_ch(pfx))
        k = _ch(kind)
        if k == 'G':
            M = sl.Matrix(m, n, nb=nb, p=p, q=q, dtype=dt, device=dev)
        elif k in ('L', 'U'):
            M = sl.HermitianMatrix(sl.Uplo.Lower if k == 'L' else sl.Uplo.Upper, n, nb=nb, p=p, q=q, dtype=dt,
                                   device=dev)
        else:
            raise ValueError(k)
        M.insertLocalTiles(device=dev.index if dev.type == "cuda" else -1)
        return _put(M)
    if op == "destroy":
        _H.pop(args[0], None)
        return 0
    if op == "pivots_create":
        return _put(sl.Pivots())
    if op == "local_size":
        lb = _H[args[0]].local_block()
        return lb.mloc * 1000000000 + lb.nloc
    if op in ("get_local", "set_local"):
        h, ptr, ld = args
        M = _H[h]
        lb = M.local_block()
        pfx = {torch.float32: 's', torch.float64: 'd', torch.complex64: 'c', torch.complex128: 'z'}[M.storage.dtype]
        if lb.mloc == 0 or lb.nloc == 0:
            return 0
        host = torch.from_numpy(_arr(pfx, ptr, lb.mloc, lb.nloc, ld)).as_strided((lb.mloc, lb.nloc), (1, ld))
        if op == "get_local":
            host.copy_(lb.data.cpu())
        else:
            lb.data.copy_(host.to(lb.data.device))
            M.storage.mark_local_modified(M.storage.origin_slot)
        return 0
    if op == "generate":
        h, kind, seed = args
        sl.generate_matrix(_H[h], {0: "rands", 1: "poev", 2: "randn"}[kind], seed)
        return 0
    if op == "norm":
        h, nrm = args
        return float(sl.norm(sl.Norm.from_string(_ch(nrm)), _H[h]))
    if op == "gemm":
        al, ha, hb, be, hc = args
        sl.gemm(al, _H[ha], _H[hb], be, _H[hc], _OPTS)
        return 0
    if op == "potrf":
        return sl.potrf(_herm(sl, args[0]), _OPTS)
    if op == "posv":
        return sl.posv(_herm(sl, args[0]), _H[args[1]], _OPTS)
    if op == "getrf":
        return sl.getrf(_H[args[0]], _H[args[1]], _OPTS)
    if op == "getrs":
        sl.getrs(_H[args[0]], _H[args[1]], _H[args[2]], _OPTS)
        return 0
    if op == "gesv":
        ha, hp, hb = args
        return sl.gesv(_H[ha], _H[hp], _H[hb], _OPTS)
    if op == "geqrf_gels":
        ha, hb = args
        return sl.gels(_H[ha], sl.TriangularFactors(), _H[hb], _OPTS)
    if op == "heev":
        ha, wptr, hz = args
        w = sl.heev(_H[ha], None, _H[hz] if hz else None, _OPTS)
        _put_reals(wptr, w)
        return 0
    return _handle_more(sl, op, *args)


# ---- options and the wider routine set of the handle API (C++ header
# include/slate_amd/slate_amd.hh wraps these; SLATE's C API: one
# slate_<routine>_c<type> per routine, src/c_api/wrappers.cc)
_OPTS = {}


def _put_reals(ptr, v):
    n = v.numel()
    if n:
        np.ctypeslib.as_array((ctypes.c_double * n).from_address(ptr))[:] = v.real.double().cpu().numpy()


def _tri(sl, h, uplo, diag):
    """Triangular view (uplo, diag) of a handle's matrix; an op'd view keeps its op."""
    M = _H[h]
    return sl.TriangularMatrix(sl.Uplo(_ch(uplo)), matrix=M, diag=sl.Diag(_ch(diag)))


def _herm(sl, h):
    M = _H[h]
    return M if isinstance(M, sl.HermitianMatrix) else sl.HermitianMatrix(sl.Uplo.Lower, matrix=M)


def _handle_more(sl, op, *args):
    if op == "set_option":
        name, value = args
        from ..core.options import _TYPES, _normalize_key
        key = _normalize_key(name)
        if key in _TYPES:
            _OPTS[key] = _TYPES[key].from_string(value)
        else:
            v = value.strip().lower()
            if v in ("true", "false"):
                _OPTS[key] = v == "true"
            else:
                try:
                    _OPTS[key] = int(v)
                except ValueError:
                    _OPTS[key] = float(v)
        return 0
    if op == "clear_options":
        _OPTS.clear()
        return 0
    if op == "sub":
        h, i1, i2, j1, j2 = args
        return _put(_H[h].sub(i1, i2, j1, j2))
    if op == "op_view":
        h, t = args
        M = _H[h]
        return _put(M.conj_transpose() if _ch(t) == 'C' else M.transpose())
    if op == "dims":
        M = _H[args[0]]
        return M.m() * 1000000000 + M.n()
    if op == "tiles":
        M = _H[args[0]]
        return M.mt() * 1000000000 + M.nt()
    if op == "tfactors_create":
        return _put(sl.TriangularFactors())
    if op in ("trsm", "trmm"):
        side, uplo, diag, al, ha, hb = args
        getattr(sl, op)(sl.Side(_ch(side)), al, _tri(sl, ha, uplo, diag), _H[hb], _OPTS)
        return 0
    if op == "herk":
        al, ha, be, hc = args
        sl.herk(al, _H[ha], be, _herm(sl, hc), _OPTS)
        return 0
    if op == "her2k":
        al, ha, hb, be, hc = args
        sl.her2k(al, _H[ha], _H[hb], be, _herm(sl, hc), _OPTS)
        return 0
    if op == "hemm":
        side, al, ha, hb, be, hc = args
        sl.hemm(sl.Side(_ch(side)), al, _herm(sl, ha), _H[hb], be, _H[hc], _OPTS)
        return 0
    if op == "potrs":
        sl.potrs(_herm(sl, args[0]), _H[args[1]], _OPTS)
        return 0
    if op == "potri":
        return sl.potri(_herm(sl, args[0]), _OPTS)
    if op == "trtri":
        uplo, diag, ha = args
        return sl.trtri(_tri(sl, ha, uplo, diag), _OPTS)
    if op == "getri":
        return sl.getri(_H[args[0]], _H[args[1]], _OPTS)
    if op in ("geqrf", "gelqf"):
        return getattr(sl, op)(_H[args[0]], _H[args[1]], _OPTS)
    if op in ("unmqr", "unmlq"):
        side, o, ha, ht, hc = args
        getattr(sl, op)(sl.Side(_ch(side)), sl.Op(_ch(o)), _H[ha], _H[ht], _H[hc], _OPTS)
        return 0
    if op == "gels_t":
        ha, ht, hb = args
        return sl.gels(_H[ha], _H[ht], _H[hb], _OPTS)
    if op == "hesv":
        ha, hb = args
        return sl.hesv(_herm(sl, ha), B=_H[hb], opts=_OPTS)
    if op in ("gesv_mixed", "posv_mixed", "gesv_mixed_gmres", "posv_mixed_gmres"):
        if op.startswith("gesv"):
            ha, hp, hb, hx, itp = args
            r = getattr(sl, op)(_H[ha], _H[hp], _H[hb], _H[hx], _OPTS)
        else:
            ha, hb, hx, itp = args
            r = getattr(sl, op)(_herm(sl, ha), _H[hb], _H[hx], _OPTS)
        info, it = (r if isinstance(r, tuple) else (r, 0))
        if itp:
            _iarr(itp, 1)[0] = int(it)
        return int(info)
    if op in ("gesv_rbt", "gesv_nopiv"):
        return getattr(sl, op)(_H[args[0]], _H[args[1]], _OPTS)
    if op == "svd_vals":
        ha, sptr = args
        _put_reals(sptr, sl.svd_vals(_H[ha], None, _OPTS))
        return 0
    if op == "hegv":
        it, ha, hb, wptr, hz = args
        w = sl.hegv(it, _herm(sl, ha), _herm(sl, hb), None, _H[hz] if hz else None, _OPTS)
        _put_reals(wptr, w)
        return 0
    if op == "add":
        al, ha, be, hb = args
        sl.add(al, _H[ha], be, _H[hb], _OPTS)
        return 0
    if op == "copy":
        sl.copy(_H[args[0]], _H[args[1]], _OPTS)
        return 0
    if op == "scale":
        num, den, ha = args
        sl.scale(num, den, _H[ha], _OPTS)
        return 0
    if op == "set":
        off, dg, ha = args
        sl.set(off, dg, _H[ha], _OPTS)
        return 0
    if op == "gecondest":
        nrm, ha, hp, anorm = args
        return float(sl.gecondest(sl.Norm.from_string(_ch(nrm)), _H[ha], _H[hp], anorm, _OPTS))
    if op == "pocondest":
        nrm, ha, anorm = args
        return float(sl.pocondest(sl.Norm.from_string(_ch(nrm)), _herm(sl, ha), anorm, _OPTS))
    raise ValueError(op)
