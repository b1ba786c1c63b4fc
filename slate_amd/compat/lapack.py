"""LAPACK-style API: `slate_amd.compat.lapack.dpotrf(uplo, n, a, lda)` etc.

Reference: `lapack_api/` (SLATE_xPOTRF-style Fortran-callable wrappers
building `fromLAPACK` matrices on a 1x1 grid, env SLATE_LAPACK_TARGET /
NB / IB / VERBOSE, `lapack_api/lapack_slate.hh:24-95`).

Here the routines take column-major arrays (numpy arrays or torch tensors,
host or device) with LAPACK argument order and return LAPACK's `info`
(plus the usual outputs).  Host arrays are staged to the GPU when the
target is "devices" (default if a GPU is present; override with
SLATE_AMD_LAPACK_TARGET=host|devices, tile size SLATE_AMD_LAPACK_NB,
default 512 on devices / 256 on the host).  The C ABI in
csrc/capi exports the same routines as `slate_<x><routine>_`.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .. import ops
from ..core.enums import Diag, Norm, Op, Option, Side, Target, Uplo
from ..core.matrix import (HermitianMatrix, Matrix, Pivots, SymmetricMatrix, TriangularFactors,
                           TriangularMatrix)

_PFX = {'s': torch.float32, 'd': torch.float64, 'c': torch.complex64, 'z': torch.complex128}


def _target():
    t = os.environ.get("SLATE_AMD_LAPACK_TARGET", "").lower()
    if t in ("host", "hosttask", "cpu"):
        return "host"
    return "devices" if torch.cuda.is_available() else "host"


def _nb():
    v = os.environ.get("SLATE_AMD_LAPACK_NB")
    if v:
        return int(v)
    return 512 if _target() == "devices" else 256


def _verbose(name, *dims):
    if os.environ.get("SLATE_AMD_LAPACK_VERBOSE", "0") not in ("0", ""):
        print(f"slate_amd.lapack {name} {dims} target={_target()}", flush=True)


class _Arr:
    """Column-major working copy of a user array.  1-D arrays are flat
    Fortran storage with leading dimension lda; 2-D arrays (numpy or torch,
    any memory order) are the matrix itself.  writeback() stores the result
    into the user's array."""

    def __init__(self, a, rows, cols, lda, dtype):
        t = torch.from_numpy(a) if isinstance(a, np.ndarray) else a
        if t.dim() == 1:
            lda = max(1, lda, rows)
            need = lda * max(cols - 1, 0) + rows if cols > 0 and rows > 0 else 0
            if t.numel() < need:
                raise ValueError(f"array too small: {t.numel()} < {need}")
            self.user = t.as_strided((rows, cols), (1, lda)) if need else t[:0].reshape(0, 0)
        else:
            self.user = t[:rows, :cols]
        dev = torch.device("cuda") if _target() == "devices" else t.device
        self.view = ops.colmajor_empty(rows, cols, dtype, dev)
        if rows and cols:
            self.view.copy_(self.user)
        self.rows, self.cols = rows, cols
        self.ld = max(1, self.view.stride(1)) if cols > 1 else max(1, rows)

    @property
    def work(self):
        return self.view

    @property
    def lda(self):
        return self.ld

    def writeback(self):
        if self.rows and self.cols:
            self.user.copy_(self.view.to(self.user.device).to(self.user.dtype))


def _M(arr, m, n):
    return Matrix.fromLAPACK(m, n, arr.work, arr.lda, nb=_nb(), comm=_self())


def _self():
    """LAPACK-style calls are per process (the reference builds them on
    MPI_COMM_SELF, lapack_api/lapack_slate.hh): never a collective."""
    from ..parallel.comm import self_comm
    return self_comm()


def _opts():
    return {Option.Target: Target.Devices if _target() == "devices" else Target.HostTask}


def _uplo(u):
    return Uplo.Lower if str(u).upper().startswith('L') else Uplo.Upper


def _op(t):
    t = str(t).upper()[0]
    return Op.NoTrans if t == 'N' else (Op.Trans if t == 'T' else Op.ConjTrans)


def _make(pfx):
    dt = _PFX[pfx]
    real = not dt.is_complex
    g = {}

    def gemm(transa, transb, m, n, k, alpha, a, lda, b, ldb, beta, c, ldc):
        _verbose(pfx + "gemm", m, n, k)
        from ..models.blas3 import gemm as _g
        ta, tb = _op(transa), _op(transb)
        A = _Arr(a, m if ta == Op.NoTrans else k, k if ta == Op.NoTrans else m, lda, dt)
        B = _Arr(b, k if tb == Op.NoTrans else n, n if tb == Op.NoTrans else k, ldb, dt)
        C = _Arr(c, m, n, ldc, dt)
        MA = _M(A, A.rows, A.cols)
        MB = _M(B, B.rows, B.cols)
        MA = MA if ta == Op.NoTrans else (MA.transpose() if ta == Op.Trans else MA.conj_transpose())
        MB = MB if tb == Op.NoTrans else (MB.transpose() if tb == Op.Trans else MB.conj_transpose())
        _g(alpha, MA, MB, beta, _M(C, m, n), _opts())
        C.writeback()
        return 0
    g["gemm"] = gemm

    def potrf(uplo, n, a, lda):
        _verbose(pfx + "potrf", n)
        from ..models.chol import potrf as _p
        A = _Arr(a, n, n, lda, dt)
        H = HermitianMatrix.fromLAPACK(_uplo(uplo), n, A.work, A.lda, nb=_nb(), comm=_self())
        info = _p(H, _opts())
        A.writeback()
        return info
    g["potrf"] = potrf

    def potrs(uplo, n, nrhs, a, lda, b, ldb):
        from ..models.chol import potrs as _p
        A = _Arr(a, n, n, lda, dt)
        B = _Arr(b, n, nrhs, ldb, dt)
        H = HermitianMatrix.fromLAPACK(_uplo(uplo), n, A.work, A.lda, nb=_nb(), comm=_self())
        _p(H, _M(B, n, nrhs), _opts())
        B.writeback()
        return 0
    g["potrs"] = potrs

    def posv(uplo, n, nrhs, a, lda, b, ldb):
        info = potrf(uplo, n, a, lda)
        if info == 0:
            potrs(uplo, n, nrhs, a, lda, b, ldb)
        return info
    g["posv"] = posv

    def potri(uplo, n, a, lda):
        from ..models.chol import potri as _p
        A = _Arr(a, n, n, lda, dt)
        H = HermitianMatrix.fromLAPACK(_uplo(uplo), n, A.work, A.lda, nb=_nb(), comm=_self())
        info = _p(H, _opts())
        A.writeback()
        return info
    g["potri"] = potri

    def getrf(m, n, a, lda, ipiv):
        """ipiv: int array (1-based on return, LAPACK convention)."""
        _verbose(pfx + "getrf", m, n)
        from ..models.lu import getrf as _g
        A = _Arr(a, m, n, lda, dt)
        piv = Pivots()
        info = _g(_M(A, m, n), piv, _opts())
        A.writeback()
        p = (piv.ipiv.cpu() + 1).numpy()
        ip = ipiv if isinstance(ipiv, np.ndarray) else None
        if ip is not None:
            ip[:len(p)] = p
        else:
            ipiv[:len(p)] = torch.from_numpy(p).to(ipiv.device, ipiv.dtype)
        return info
    g["getrf"] = getrf

    def getrs(trans, n, nrhs, a, lda, ipiv, b, ldb):
        from ..models.lu import getrs as _g
        A = _Arr(a, n, n, lda, dt)
        B = _Arr(b, n, nrhs, ldb, dt)
        ip = torch.as_tensor(np.asarray(ipiv) if isinstance(ipiv, np.ndarray) else ipiv.cpu()).to(torch.int64)[:n] - 1
        piv = Pivots()
        piv.set(ip, _nb())
        MA = _M(A, n, n)
        t = _op(trans)
        MA = MA if t == Op.NoTrans else (MA.transpose() if t == Op.Trans else MA.conj_transpose())
        _g(MA, piv, _M(B, n, nrhs), _opts())
        B.writeback()
        return 0
    g["getrs"] = getrs

    def gesv(n, nrhs, a, lda, ipiv, b, ldb):
        info = getrf(n, n, a, lda, ipiv)
        if info == 0:
            getrs('N', n, nrhs, a, lda, ipiv, b, ldb)
        return info
    g["gesv"] = gesv

    def trsm(side, uplo, transa, diag, m, n, alpha, a, lda, b, ldb):
        from ..models.blas3 import trsm as _t
        k = m if str(side).upper()[0] == 'L' else n
        A = _Arr(a, k, k, lda, dt)
        B = _Arr(b, m, n, ldb, dt)
        T = TriangularMatrix.fromLAPACK(_uplo(uplo), Diag.Unit if str(diag).upper()[0] == 'U' else Diag.NonUnit,
                                        k, A.work, A.lda, nb=_nb(), comm=_self())
        t = _op(transa)
        T = T if t == Op.NoTrans else (T.transpose() if t == Op.Trans else T.conj_transpose())
        _t(Side.Left if str(side).upper()[0] == 'L' else Side.Right, alpha, T, _M(B, m, n), _opts())
        B.writeback()
        return 0
    g["trsm"] = trsm

    def trmm(side, uplo, transa, diag, m, n, alpha, a, lda, b, ldb):
        from ..models.blas3 import trmm as _t
        k = m if str(side).upper()[0] == 'L' else n
        A = _Arr(a, k, k, lda, dt)
        B = _Arr(b, m, n, ldb, dt)
        T = TriangularMatrix.fromLAPACK(_uplo(uplo), Diag.Unit if str(diag).upper()[0] == 'U' else Diag.NonUnit,
                                        k, A.work, A.lda, nb=_nb(), comm=_self())
        t = _op(transa)
        T = T if t == Op.NoTrans else (T.transpose() if t == Op.Trans else T.conj_transpose())
        _t(Side.Left if str(side).upper()[0] == 'L' else Side.Right, alpha, T, _M(B, m, n), _opts())
        B.writeback()
        return 0
    g["trmm"] = trmm

    def herk(uplo, trans, n, k, alpha, a, lda, beta, c, ldc):
        from ..models.blas3 import herk as _h, syrk as _s
        t = _op(trans)
        A = _Arr(a, n if t == Op.NoTrans else k, k if t == Op.NoTrans else n, lda, dt)
        C = _Arr(c, n, n, ldc, dt)
        MA = _M(A, A.rows, A.cols)
        MA = MA if t == Op.NoTrans else MA.conj_transpose() if not real or t == Op.ConjTrans else MA.transpose()
        H = HermitianMatrix.fromLAPACK(_uplo(uplo), n, C.work, C.lda, nb=_nb(), comm=_self())
        (_h if (not real or True) else _s)(alpha, MA, beta, H, _opts())
        C.writeback()
        return 0

    def geqrf(m, n, a, lda, tau):
        from ..models.qr import geqrf as _q
        A = _Arr(a, m, n, lda, dt)
        T = TriangularFactors()
        _q(_M(A, m, n), T, _opts())
        A.writeback()
        taus = torch.cat([p["tau"].cpu() for p in T]) if len(T) else torch.zeros(0, dtype=dt)
        if isinstance(tau, np.ndarray):
            tau[:taus.numel()] = taus.numpy()
        else:
            tau[:taus.numel()] = taus.to(tau.device)
        return 0
    g["geqrf"] = geqrf

    def gels(trans, m, n, nrhs, a, lda, b, ldb):
        from ..models.qr import gels as _g
        A = _Arr(a, m, n, lda, dt)
        B = _Arr(b, max(m, n), nrhs, ldb, dt)
        MA = _M(A, m, n)
        t = _op(trans)
        MA = MA if t == Op.NoTrans else MA.conj_transpose()
        _g(MA, TriangularFactors(), _M(B, max(m, n), nrhs), _opts())
        B.writeback()
        return 0
    g["gels"] = gels

    def heev(jobz, uplo, n, a, lda, w):
        from ..models.eig import heev as _h
        A = _Arr(a, n, n, lda, dt)
        H = HermitianMatrix.fromLAPACK(_uplo(uplo), n, A.work, A.lda, nb=_nb(), comm=_self())
        Z = None
        if str(jobz).upper()[0] == 'V':
            Z = Matrix(n, n, nb=_nb(), comm=_self(), dtype=dt, device=A.work.device)
            Z.insertLocalTiles(device=A.work.device.index if A.work.is_cuda else -1)
        vals = _h(H, None, Z, _opts())
        if Z is not None:
            from ..models.aux import allgather_dense
            A.view.copy_(allgather_dense(Z).to(A.view.device))
        A.writeback()
        if isinstance(w, np.ndarray):
            w[:n] = vals.cpu().numpy()
        else:
            w[:n] = vals.to(w.device, w.dtype)
        return 0
    g["heev" if not real else "syev"] = heev

    def gesvd(jobu, jobvt, m, n, a, lda, s, u, ldu, vt, ldvt):
        from ..models.svd import svd as _s
        from ..models.aux import allgather_dense
        A = _Arr(a, m, n, lda, dt)
        k = min(m, n)
        want = str(jobu).upper()[0] in 'AS' or str(jobvt).upper()[0] in 'AS'
        U = VH = None
        dev = A.work.device
        di = dev.index if dev.type == "cuda" else -1
        if str(jobu).upper()[0] in 'AS':
            U = Matrix(m, k, nb=_nb(), comm=_self(), dtype=dt, device=dev)
            U.insertLocalTiles(device=di)
        if str(jobvt).upper()[0] in 'AS':
            VH = Matrix(k, n, nb=_nb(), comm=_self(), dtype=dt, device=dev)
            VH.insertLocalTiles(device=di)
        sv = _s(_M(A, m, n), None, U, VH, _opts())
        if U is not None:
            Ua = _Arr(u, m, k, ldu, dt)
            Ua.view.copy_(allgather_dense(U).to(Ua.view.device))
            Ua.writeback()
        if VH is not None:
            Va = _Arr(vt, k, n, ldvt, dt)
            Va.view.copy_(allgather_dense(VH).to(Va.view.device))
            Va.writeback()
        if isinstance(s, np.ndarray):
            s[:k] = sv.cpu().numpy()
        else:
            s[:k] = sv.to(s.device, s.dtype)
        del want
        return 0
    g["gesvd"] = gesvd

    def lange(norm, m, n, a, lda):
        from ..models.aux import norm as _n
        A = _Arr(a, m, n, lda, dt)
        return float(_n(Norm.from_string(str(norm)), _M(A, m, n)))
    g["lange"] = lange

    # ---- BLAS-3 on symmetric / Hermitian operands (lapack_api/lapack_hemm.cc,
    #      lapack_symm.cc, lapack_her2k.cc, lapack_syr2k.cc, lapack_syrk.cc)
    def _side(sd):
        return Side.Left if str(sd).upper()[0] == 'L' else Side.Right

    def _hsmm(herm):
        def mm(side, uplo, m, n, alpha, a, lda, b, ldb, beta, c, ldc):
            from ..models.blas3 import hemm as _h, symm as _s
            k = m if _side(side) == Side.Left else n
            A = _Arr(a, k, k, lda, dt)
            B = _Arr(b, m, n, ldb, dt)
            C = _Arr(c, m, n, ldc, dt)
            cls = HermitianMatrix if herm else SymmetricMatrix
            H = cls.fromLAPACK(_uplo(uplo), k, A.work, A.lda, nb=_nb(), comm=_self())
            (_h if herm else _s)(_side(side), alpha, H, _M(B, m, n), beta, _M(C, m, n), _opts())
            C.writeback()
            return 0
        return mm
    g["hemm"] = _hsmm(True)
    g["symm"] = _hsmm(False)

    def _rk(herm):
        def rk(uplo, trans, n, k, alpha, a, lda, beta, c, ldc):
            from ..models.blas3 import herk as _h, syrk as _s
            t = _op(trans)
            A = _Arr(a, n if t == Op.NoTrans else k, k if t == Op.NoTrans else n, lda, dt)
            C = _Arr(c, n, n, ldc, dt)
            MA = _M(A, A.rows, A.cols)
            if t != Op.NoTrans:
                MA = MA.conj_transpose() if herm else MA.transpose()
            cls = HermitianMatrix if herm else SymmetricMatrix
            H = cls.fromLAPACK(_uplo(uplo), n, C.work, C.lda, nb=_nb(), comm=_self())
            (_h if herm else _s)(alpha, MA, beta, H, _opts())
            C.writeback()
            return 0
        return rk
    g["herk"] = _rk(True)
    g["syrk"] = _rk(False)

    def _r2k(herm):
        def r2k(uplo, trans, n, k, alpha, a, lda, b, ldb, beta, c, ldc):
            from ..models.blas3 import her2k as _h, syr2k as _s
            t = _op(trans)
            r, cc = (n, k) if t == Op.NoTrans else (k, n)
            A = _Arr(a, r, cc, lda, dt)
            B = _Arr(b, r, cc, ldb, dt)
            C = _Arr(c, n, n, ldc, dt)
            MA, MB = _M(A, r, cc), _M(B, r, cc)
            if t != Op.NoTrans:
                MA = MA.conj_transpose() if herm else MA.transpose()
                MB = MB.conj_transpose() if herm else MB.transpose()
            cls = HermitianMatrix if herm else SymmetricMatrix
            H = cls.fromLAPACK(_uplo(uplo), n, C.work, C.lda, nb=_nb(), comm=_self())
            (_h if herm else _s)(alpha, MA, MB, beta, H, _opts())
            C.writeback()
            return 0
        return r2k
    g["her2k"] = _r2k(True)
    g["syr2k"] = _r2k(False)

    # ---- inverses, mixed precision, eigenvalues (lapack_getri.cc,
    #      lapack_gesv_mixed.cc, lapack_heevd.cc)
    def getri(n, a, lda, ipiv):
        """Inverse from getrf's factors; ipiv 1-based (LAPACK)."""
        from ..models.lu import getri as _g
        A = _Arr(a, n, n, lda, dt)
        ip = torch.as_tensor(np.asarray(ipiv) if isinstance(ipiv, np.ndarray) else ipiv.cpu()).to(torch.int64)[:n] - 1
        piv = Pivots()
        piv.set(ip, _nb())
        info = _g(_M(A, n, n), piv, _opts())
        A.writeback()
        return info
    g["getri"] = getri

    if pfx in "dz":
        def gesv_mixed(n, nrhs, a, lda, ipiv, b, ldb, x, ldx):
            """LAPACK dsgesv / zcgesv: returns (info, iter) -- iter < 0 means
            the refinement fell back to full precision."""
            from ..models.mixed import gesv_mixed as _g
            A = _Arr(a, n, n, lda, dt)
            B = _Arr(b, n, nrhs, ldb, dt)
            X = _Arr(x, n, nrhs, ldx, dt)
            piv = Pivots()
            info, it = _g(_M(A, n, n), piv, _M(B, n, nrhs), _M(X, n, nrhs), _opts())
            X.writeback()
            p = (piv.ipiv.cpu() + 1).numpy()
            if isinstance(ipiv, np.ndarray):
                ipiv[:len(p)] = p
            else:
                ipiv[:len(p)] = torch.from_numpy(p).to(ipiv.device, ipiv.dtype)
            return info, it
        g["gesv_mixed"] = gesv_mixed

    # ---- norms of structured matrices (lapack_lanhe.cc, lapack_lansy.cc,
    #      lapack_lantr.cc)
    def _lan_sym(herm):
        def lan(norm, uplo, n, a, lda):
            from ..models.aux import norm as _n
            A = _Arr(a, n, n, lda, dt)
            cls = HermitianMatrix if herm else SymmetricMatrix
            return float(_n(Norm.from_string(str(norm)), cls.fromLAPACK(_uplo(uplo), n, A.work, A.lda, nb=_nb(), comm=_self())))
        return lan
    g["lanhe"] = _lan_sym(True)
    g["lansy"] = _lan_sym(False)

    def lantr(norm, uplo, diag, m, n, a, lda):
        from ..models.aux import norm as _n
        from ..core.matrix import TrapezoidMatrix
        A = _Arr(a, m, n, lda, dt)
        T = TrapezoidMatrix.fromLAPACK(_uplo(uplo), m, n, A.work, A.lda, nb=_nb(), comm=_self(),
                                       diag=Diag.Unit if str(diag).upper()[0] == 'U' else Diag.NonUnit)
        return float(_n(Norm.from_string(str(norm)), T))
    g["lantr"] = lantr

    # ---- condition estimates (lapack_gecon.cc, lapack_pocon.cc, lapack_trcon.cc):
    #      return (info, rcond)
    def gecon(norm, n, a, lda, anorm):
        """a holds getrf's factors with the pivots applied (LAPACK gecon
        takes no pivots: the estimate needs only the L and U solves)."""
        from ..models.condest import gecondest as _g
        A = _Arr(a, n, n, lda, dt)
        piv = Pivots()
        piv.set(torch.arange(n, dtype=torch.int64), _nb())
        return 0, float(_g(Norm.from_string(str(norm)), _M(A, n, n), piv, anorm, _opts()))
    g["gecon"] = gecon

    def pocon(uplo, n, a, lda, anorm):
        from ..models.condest import pocondest as _p
        A = _Arr(a, n, n, lda, dt)
        H = HermitianMatrix.fromLAPACK(_uplo(uplo), n, A.work, A.lda, nb=_nb(), comm=_self())
        return 0, float(_p(Norm.One, H, anorm, _opts()))
    g["pocon"] = pocon

    def trcon(norm, uplo, diag, n, a, lda):
        from ..models.condest import trcondest as _t
        A = _Arr(a, n, n, lda, dt)
        T = TriangularMatrix.fromLAPACK(_uplo(uplo), Diag.Unit if str(diag).upper()[0] == 'U' else Diag.NonUnit,
                                        n, A.work, A.lda, nb=_nb(), comm=_self())
        return 0, float(_t(Norm.from_string(str(norm)), T, None, _opts()))
    g["trcon"] = trcon

    def heevd(jobz, uplo, n, a, lda, w):
        """Divide and conquer is heev's default method (MethodEig.DC)."""
        return heev(jobz, uplo, n, a, lda, w)
    g["heevd" if not real else "syevd"] = heevd

    def trtri(uplo, diag, n, a, lda):
        from ..models.inverse import trtri as _t
        A = _Arr(a, n, n, lda, dt)
        T = TriangularMatrix.fromLAPACK(_uplo(uplo), Diag.Unit if str(diag).upper()[0] == 'U' else Diag.NonUnit,
                                        n, A.work, A.lda, nb=_nb(), comm=_self())
        info = _t(T, _opts())
        A.writeback()
        return info
    g["trtri"] = trtri

    return g


def _install():
    mod = globals()
    for pfx in _PFX:
        for name, fn in _make(pfx).items():
            fn.__name__ = pfx + name
            fn.__qualname__ = pfx + name
            mod[pfx + name] = fn


_install()
