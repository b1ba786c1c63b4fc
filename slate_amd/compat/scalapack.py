"""ScaLAPACK-style API: `pdpotrf(uplo, n, a, ia, ja, desca)` etc. on this
rank's ScaLAPACK local arrays.

Reference: `scalapack_api/` (`pdpotrf_`-style interposers that wrap the
user's ScaLAPACK arrays with `fromScaLAPACK` + BLACS grid info, env
SLATE_SCALAPACK_TARGET / LOOKAHEAD / VERBOSE,
`scalapack_api/scalapack_slate.hh:30-131`).

There is no MPI/BLACS here: the process grid comes from
`blacs_gridinit(p, q, order)` over the torch.distributed world (RCCL on
GPUs), which returns a context id used in descriptor slot 1.  Descriptors
follow ScaLAPACK: desc = [dtype, ctxt, m, n, mb, nb, rsrc, csrc, lld].
Local arrays (numpy or torch, host or device) are wrapped zero-copy when
already on the target device; host arrays are staged to the rank's GPU
for Target=devices (SLATE_AMD_SCALAPACK_TARGET=host|devices).  Global
sub-matrix offsets ia, ja (1-based) may be anything: a sub-matrix that does
not start on a tile corner is moved into an aligned work matrix on the same
grid by the piece-level redistribution (`parallel/redist.py`: each element
moves at most once, nothing is gathered) and moved back afterwards.
rsrc = csrc = 0.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..core.enums import Diag, GridOrder, Norm, Op, Option, Side, Target, Uplo
from ..core.exceptions import SlateError
from ..core.matrix import (HermitianMatrix, Matrix, Pivots, SymmetricMatrix, TrapezoidMatrix, TriangularFactors,
                           TriangularMatrix)
from ..parallel import comm as _comm

_PFX = {'s': torch.float32, 'd': torch.float64, 'c': torch.complex64, 'z': torch.complex128}
_CTX = {}


def blacs_gridinit(p, q, order="C"):
    """Create a p x q process-grid context over the world communicator."""
    world = _comm.world()
    if p * q != world.size:
        raise SlateError(f"grid {p}x{q} does not match world size {world.size}")
    ctxt = len(_CTX) + 1
    _CTX[ctxt] = (p, q, GridOrder.from_string(order) if isinstance(order, str) else order)
    return ctxt


def blacs_gridinfo(ctxt):
    p, q, order = _CTX[ctxt]
    r = _comm.world().rank
    pr, pc = (r % p, r // p) if order == GridOrder.Col else (r // q, r % q)
    return p, q, pr, pc


def numroc(n, nb, iproc, isrcproc, nprocs):
    from ..core.storage import numroc as _n
    return _n(n, nb, (iproc - isrcproc) % nprocs, nprocs)


def _target():
    t = os.environ.get("SLATE_AMD_SCALAPACK_TARGET", "").lower()
    if t in ("host", "cpu"):
        return "host"
    return "devices" if torch.cuda.is_available() else "host"


def _opts():
    la = int(os.environ.get("SLATE_AMD_SCALAPACK_LOOKAHEAD", "1"))
    return {Option.Target: Target.Devices if _target() == "devices" else Target.HostTask, Option.Lookahead: la}


class _Loc:
    """This rank's local array (lld x nloc) staged to the target device."""

    def __init__(self, a, desc, dtype):
        _, ctxt, m, n, mb, nb, rsrc, csrc, lld = [int(x) for x in desc[:9]]
        if rsrc or csrc:
            raise SlateError("scalapack: rsrc = csrc = 0 required")
        p, q, pr, pc = blacs_gridinfo(ctxt)
        self.m, self.n, self.mb, self.nb, self.p, self.q = m, n, mb, nb, p, q
        self.order = _CTX[ctxt][2]
        nloc = numroc(n, nb, pc, 0, q)
        t = torch.from_numpy(a) if isinstance(a, np.ndarray) else a
        mloc = numroc(m, mb, pr, 0, p)
        if nloc == 0 or t.numel() == 0:
            t = torch.zeros((0, max(1, lld, mloc)), dtype=t.dtype, device=t.device).t()
        flat = t.reshape(-1) if t.dim() == 1 else t.t().reshape(-1) if t.stride(0) != 1 else None
        if t.dim() == 2 and t.stride(0) == 1:
            self.user = t[:, :nloc]
            lld = max(1, t.stride(1))
        else:
            lld = max(1, lld)
            self.user = flat.as_strided((lld, nloc), (1, lld)) if nloc else flat[:0].reshape(0, 0)
        dev = torch.device("cuda", torch.cuda.current_device()) if _target() == "devices" else t.device
        if self.user.device == dev and self.user.dtype == dtype:
            self.work = self.user
            self.copy = False
        else:
            from .. import ops
            self.work = ops.colmajor_empty(lld, nloc, dtype, dev)
            if nloc:
                self.work.copy_(self.user)
            self.copy = True
        self.lld = lld

    def matrix(self, kind=Matrix, **kw):
        comm = _comm.world()
        if kind is Matrix:
            return Matrix.fromScaLAPACK(self.m, self.n, self.work, self.lld, self.mb, self.nb, self.order,
                                        self.p, self.q, comm)
        if kind is HermitianMatrix:
            return HermitianMatrix.fromScaLAPACK(kw["uplo"], self.n, self.work, self.lld, self.nb, self.p,
                                                 self.q, comm, order=self.order)
        if kind is TriangularMatrix:
            return TriangularMatrix.fromScaLAPACK(kw["uplo"], kw["diag"], self.n, self.work, self.lld, self.nb,
                                                  self.p, self.q, comm, order=self.order)
        if kind is SymmetricMatrix:
            return SymmetricMatrix.fromScaLAPACK(kw["uplo"], self.n, self.work, self.lld, self.nb, self.p,
                                                 self.q, comm, order=self.order)
        if kind is TrapezoidMatrix:
            M = Matrix.fromScaLAPACK(self.m, self.n, self.work, self.lld, self.mb, self.nb, self.order,
                                     self.p, self.q, comm)
            return TrapezoidMatrix(kw["uplo"], matrix=M, diag=kw["diag"])
        raise SlateError("bad kind")

    def writeback(self):
        if self.copy and self.user.numel():
            self.user.copy_(self.work.to(self.user.device).to(self.user.dtype))


def _sub(L, ia, ja, m, n, kind=Matrix, **kw):
    """The (m x n) global sub-matrix at 1-based (ia, ja) of the ScaLAPACK
    array L as a driver-ready matrix of ``kind``, and a finisher that moves
    an aligned work copy back (no-op for whole matrices)."""
    ia, ja, m, n = int(ia), int(ja), int(m), int(n)
    if ia == 1 and ja == 1 and m == L.m and n == L.n:
        return L.matrix(kind, **kw), (lambda: None)
    from ..models.aux import copy
    full = L.matrix()
    view = full.slice(ia - 1, ia - 1 + m - 1, ja - 1, ja - 1 + n - 1)
    s = full.storage
    W = Matrix(m, n, nb=L.nb, mb=L.mb, p=L.p, q=L.q, comm=_comm.world(), dtype=s.dtype, device=s.device,
               order=L.order)
    W.insertLocalTiles(device=s.device.index if s.device.type == "cuda" else -1)
    copy(view, W)
    if kind is HermitianMatrix:
        M = HermitianMatrix(kw["uplo"], W)
    elif kind is SymmetricMatrix:
        M = SymmetricMatrix(kw["uplo"], W)
    elif kind is TriangularMatrix:
        M = TriangularMatrix(kw["uplo"], W, diag=kw["diag"])
    elif kind is TrapezoidMatrix:
        M = TrapezoidMatrix(kw["uplo"], matrix=W, diag=kw["diag"])
    else:
        M = W
    return M, (lambda: copy(W, view))


def _uplo(u):
    return Uplo.Lower if str(u).upper()[0] == 'L' else Uplo.Upper


def _op(t):
    t = str(t).upper()[0]
    return Op.NoTrans if t == 'N' else (Op.Trans if t == 'T' else Op.ConjTrans)


def _opm(M, t):
    return M if t == Op.NoTrans else (M.transpose() if t == Op.Trans else M.conj_transpose())


def _make(pfx):
    dt = _PFX[pfx]
    g = {}

    def gemm(transa, transb, m, n, k, alpha, a, ia, ja, desca, b, ib, jb, descb, beta, c, ic, jc, descc):
        from ..models.blas3 import gemm as _g
        A, B, C = _Loc(a, desca, dt), _Loc(b, descb, dt), _Loc(c, descc, dt)
        ta, tb = _op(transa), _op(transb)
        Am, _ = _sub(A, ia, ja, *((m, k) if ta == Op.NoTrans else (k, m)))
        Bm, _ = _sub(B, ib, jb, *((k, n) if tb == Op.NoTrans else (n, k)))
        Cm, done = _sub(C, ic, jc, m, n)
        _g(alpha, _opm(Am, ta), _opm(Bm, tb), beta, Cm, _opts())
        done()
        C.writeback()
        return 0
    g["gemm"] = gemm

    def potrf(uplo, n, a, ia, ja, desca):
        from ..models.chol import potrf as _p
        A = _Loc(a, desca, dt)
        Am, done = _sub(A, ia, ja, n, n, HermitianMatrix, uplo=_uplo(uplo))
        info = _p(Am, _opts())
        done()
        A.writeback()
        return info
    g["potrf"] = potrf

    def potrs(uplo, n, nrhs, a, ia, ja, desca, b, ib, jb, descb):
        from ..models.chol import potrs as _p
        A, B = _Loc(a, desca, dt), _Loc(b, descb, dt)
        Am, _ = _sub(A, ia, ja, n, n, HermitianMatrix, uplo=_uplo(uplo))
        Bm, done = _sub(B, ib, jb, n, nrhs)
        _p(Am, Bm, _opts())
        done()
        B.writeback()
        return 0
    g["potrs"] = potrs

    def posv(uplo, n, nrhs, a, ia, ja, desca, b, ib, jb, descb):
        info = potrf(uplo, n, a, ia, ja, desca)
        if info == 0:
            potrs(uplo, n, nrhs, a, ia, ja, desca, b, ib, jb, descb)
        return info
    g["posv"] = posv

    def getrf(m, n, a, ia, ja, desca, ipiv):
        """ipiv: 1-based pivots relative to the sub-matrix (length min(m, n))."""
        from ..models.lu import getrf as _g
        A = _Loc(a, desca, dt)
        Am, done = _sub(A, ia, ja, m, n)
        piv = Pivots()
        info = _g(Am, piv, _opts())
        done()
        A.writeback()
        p = (piv.ipiv.cpu() + 1)
        if isinstance(ipiv, np.ndarray):
            ipiv[:p.numel()] = p.numpy()
        else:
            ipiv[:p.numel()] = p.to(ipiv.device, ipiv.dtype)
        return info
    g["getrf"] = getrf

    def getrs(trans, n, nrhs, a, ia, ja, desca, ipiv, b, ib, jb, descb):
        from ..models.lu import getrs as _g
        A, B = _Loc(a, desca, dt), _Loc(b, descb, dt)
        ip = torch.as_tensor(np.asarray(ipiv) if isinstance(ipiv, np.ndarray) else ipiv.cpu()).to(torch.int64)
        piv = Pivots()
        piv.set(ip[:n] - 1, A.nb)
        Am, _ = _sub(A, ia, ja, n, n)
        Bm, done = _sub(B, ib, jb, n, nrhs)
        _g(_opm(Am, _op(trans)), piv, Bm, _opts())
        done()
        B.writeback()
        return 0
    g["getrs"] = getrs

    def gesv(n, nrhs, a, ia, ja, desca, ipiv, b, ib, jb, descb):
        info = getrf(n, n, a, ia, ja, desca, ipiv)
        if info == 0:
            getrs('N', n, nrhs, a, ia, ja, desca, ipiv, b, ib, jb, descb)
        return info
    g["gesv"] = gesv

    def trsm(side, uplo, transa, diag, m, n, alpha, a, ia, ja, desca, b, ib, jb, descb):
        from ..models.blas3 import trsm as _t
        A, B = _Loc(a, desca, dt), _Loc(b, descb, dt)
        left = str(side).upper()[0] == 'L'
        k = m if left else n
        T, _ = _sub(A, ia, ja, k, k, TriangularMatrix, uplo=_uplo(uplo),
                    diag=Diag.Unit if str(diag).upper()[0] == 'U' else Diag.NonUnit)
        Bm, done = _sub(B, ib, jb, m, n)
        _t(Side.Left if left else Side.Right, alpha, _opm(T, _op(transa)), Bm, _opts())
        done()
        B.writeback()
        return 0
    g["trsm"] = trsm

    def geqrf(m, n, a, ia, ja, desca, tau=None):
        from ..models.qr import geqrf as _q
        A = _Loc(a, desca, dt)
        Am, done = _sub(A, ia, ja, m, n)
        T = TriangularFactors()
        _q(Am, T, _opts())
        done()
        A.writeback()
        return T
    g["geqrf"] = geqrf

    def gels(trans, m, n, nrhs, a, ia, ja, desca, b, ib, jb, descb):
        from ..models.qr import gels as _g
        A, B = _Loc(a, desca, dt), _Loc(b, descb, dt)
        Am, done_a = _sub(A, ia, ja, m, n)
        Bm, done = _sub(B, ib, jb, max(m, n), nrhs)
        _g(_opm(Am, _op(trans)), TriangularFactors(), Bm, _opts())
        done()
        done_a()
        A.writeback()
        B.writeback()
        return 0
    g["gels"] = gels

    def lange(norm, m, n, a, ia, ja, desca):
        from ..models.aux import norm as _n
        Am, _ = _sub(_Loc(a, desca, dt), ia, ja, m, n)
        return float(_n(Norm.from_string(str(norm)), Am))
    g["lange"] = lange

    def heev(jobz, uplo, n, a, ia, ja, desca, w, z=None, iz=1, jz=1, descz=None):
        from ..models.eig import heev as _h
        A = _Loc(a, desca, dt)
        Z = _Loc(z, descz, dt) if str(jobz).upper()[0] == 'V' else None
        Am, _ = _sub(A, ia, ja, n, n, HermitianMatrix, uplo=_uplo(uplo))
        Zm, done = _sub(Z, iz, jz, n, n) if Z else (None, lambda: None)
        vals = _h(Am, None, Zm, _opts())
        done()
        if Z:
            Z.writeback()
        if isinstance(w, np.ndarray):
            w[:n] = vals.cpu().numpy()
        else:
            w[:n] = vals.to(w.device, w.dtype)
        return 0
    g["heev" if dt.is_complex else "syev"] = heev

    def gesvd(jobu, jobvt, m, n, a, ia, ja, desca, s, u=None, iu=1, ju=1, descu=None, vt=None, ivt=1, jvt=1,
              descvt=None):
        from ..models.svd import svd as _s
        if int(ia) != 1 or int(ja) != 1:
            raise SlateError("pgesvd: ia = ja = 1 required")
        A = _Loc(a, desca, dt)
        U = _Loc(u, descu, dt) if str(jobu).upper()[0] == 'V' else None
        VT = _Loc(vt, descvt, dt) if str(jobvt).upper()[0] == 'V' else None
        sv = _s(A.matrix(), None, U.matrix() if U else None, VT.matrix() if VT else None, _opts())
        for x in (U, VT):
            if x:
                x.writeback()
        k = min(m, n)
        if isinstance(s, np.ndarray):
            s[:k] = sv.cpu().numpy()
        else:
            s[:k] = sv.to(s.device, s.dtype)
        return 0
    g["gesvd"] = gesvd

    # ---- BLAS-3 (scalapack_api/scalapack_trmm.cc, _herk, _syrk, _her2k,
    #      _syr2k, _hemm, _symm)
    def _diag(d):
        return Diag.Unit if str(d).upper()[0] == 'U' else Diag.NonUnit

    def trmm(side, uplo, transa, diag, m, n, alpha, a, ia, ja, desca, b, ib, jb, descb):
        from ..models.blas3 import trmm as _t
        A, B = _Loc(a, desca, dt), _Loc(b, descb, dt)
        left = str(side).upper()[0] == 'L'
        k = m if left else n
        T, _ = _sub(A, ia, ja, k, k, TriangularMatrix, uplo=_uplo(uplo), diag=_diag(diag))
        Bm, done = _sub(B, ib, jb, m, n)
        _t(Side.Left if left else Side.Right, alpha, _opm(T, _op(transa)), Bm, _opts())
        done()
        B.writeback()
        return 0
    g["trmm"] = trmm

    def _rk(herm):
        def rk(uplo, trans, n, k, alpha, a, ia, ja, desca, beta, c, ic, jc, descc):
            from ..models.blas3 import herk as _h, syrk as _s
            A, C = _Loc(a, desca, dt), _Loc(c, descc, dt)
            t = _op(trans)
            Am, _ = _sub(A, ia, ja, *((n, k) if t == Op.NoTrans else (k, n)))
            if t != Op.NoTrans:
                Am = Am.conj_transpose() if herm else Am.transpose()
            Cm, done = _sub(C, ic, jc, n, n, HermitianMatrix if herm else SymmetricMatrix, uplo=_uplo(uplo))
            (_h if herm else _s)(alpha, Am, beta, Cm, _opts())
            done()
            C.writeback()
            return 0
        return rk
    g["herk"] = _rk(True)
    g["syrk"] = _rk(False)

    def _r2k(herm):
        def r2k(uplo, trans, n, k, alpha, a, ia, ja, desca, b, ib, jb, descb, beta, c, ic, jc, descc):
            from ..models.blas3 import her2k as _h, syr2k as _s
            A, B, C = _Loc(a, desca, dt), _Loc(b, descb, dt), _Loc(c, descc, dt)
            t = _op(trans)
            shp = (n, k) if t == Op.NoTrans else (k, n)
            Am, _ = _sub(A, ia, ja, *shp)
            Bm, _ = _sub(B, ib, jb, *shp)
            if t != Op.NoTrans:
                Am = Am.conj_transpose() if herm else Am.transpose()
                Bm = Bm.conj_transpose() if herm else Bm.transpose()
            Cm, done = _sub(C, ic, jc, n, n, HermitianMatrix if herm else SymmetricMatrix, uplo=_uplo(uplo))
            (_h if herm else _s)(alpha, Am, Bm, beta, Cm, _opts())
            done()
            C.writeback()
            return 0
        return r2k
    g["her2k"] = _r2k(True)
    g["syr2k"] = _r2k(False)

    def _mm(herm):
        def mm(side, uplo, m, n, alpha, a, ia, ja, desca, b, ib, jb, descb, beta, c, ic, jc, descc):
            from ..models.blas3 import hemm as _h, symm as _s
            A, B, C = _Loc(a, desca, dt), _Loc(b, descb, dt), _Loc(c, descc, dt)
            left = str(side).upper()[0] == 'L'
            k = m if left else n
            Am, _ = _sub(A, ia, ja, k, k, HermitianMatrix if herm else SymmetricMatrix, uplo=_uplo(uplo))
            Bm, _ = _sub(B, ib, jb, m, n)
            Cm, done = _sub(C, ic, jc, m, n)
            (_h if herm else _s)(Side.Left if left else Side.Right, alpha, Am, Bm, beta, Cm, _opts())
            done()
            C.writeback()
            return 0
        return mm
    g["hemm"] = _mm(True)
    g["symm"] = _mm(False)

    # ---- inverses (scalapack_potri.cc, scalapack_getri.cc)
    def potri(uplo, n, a, ia, ja, desca):
        from ..models.chol import potri as _p
        A = _Loc(a, desca, dt)
        Am, done = _sub(A, ia, ja, n, n, HermitianMatrix, uplo=_uplo(uplo))
        info = _p(Am, _opts())
        done()
        A.writeback()
        return info
    g["potri"] = potri

    def getri(n, a, ia, ja, desca, ipiv):
        from ..models.lu import getri as _g
        A = _Loc(a, desca, dt)
        ip = torch.as_tensor(np.asarray(ipiv) if isinstance(ipiv, np.ndarray) else ipiv.cpu()).to(torch.int64)
        piv = Pivots()
        piv.set(ip[:n] - 1, A.nb)
        Am, done = _sub(A, ia, ja, n, n)
        info = _g(Am, piv, _opts())
        done()
        A.writeback()
        return info
    g["getri"] = getri

    # ---- norms (scalapack_lanhe.cc, _lansy, _lantr)
    def _lan(herm):
        def lan(norm, uplo, n, a, ia, ja, desca):
            from ..models.aux import norm as _n
            Am, _ = _sub(_Loc(a, desca, dt), ia, ja, n, n, HermitianMatrix if herm else SymmetricMatrix,
                         uplo=_uplo(uplo))
            return float(_n(Norm.from_string(str(norm)), Am))
        return lan
    g["lanhe"] = _lan(True)
    g["lansy"] = _lan(False)

    def lantr(norm, uplo, diag, m, n, a, ia, ja, desca):
        from ..models.aux import norm as _n
        Am, _ = _sub(_Loc(a, desca, dt), ia, ja, m, n, TrapezoidMatrix, uplo=_uplo(uplo), diag=_diag(diag))
        return float(_n(Norm.from_string(str(norm)), Am))
    g["lantr"] = lantr

    # ---- condition estimates: (info, rcond) (scalapack_gecon.cc, _pocon, _trcon)
    def gecon(norm, n, a, ia, ja, desca, anorm):
        from ..models.condest import gecondest as _g
        A = _Loc(a, desca, dt)
        Am, _ = _sub(A, ia, ja, n, n)
        piv = Pivots()
        piv.set(torch.arange(n, dtype=torch.int64), A.nb)
        return 0, float(_g(Norm.from_string(str(norm)), Am, piv, anorm, _opts()))
    g["gecon"] = gecon

    def pocon(uplo, n, a, ia, ja, desca, anorm):
        from ..models.condest import pocondest as _p
        Am, _ = _sub(_Loc(a, desca, dt), ia, ja, n, n, HermitianMatrix, uplo=_uplo(uplo))
        return 0, float(_p(Norm.One, Am, anorm, _opts()))
    g["pocon"] = pocon

    def trcon(norm, uplo, diag, n, a, ia, ja, desca):
        from ..models.condest import trcondest as _t
        Am, _ = _sub(_Loc(a, desca, dt), ia, ja, n, n, TriangularMatrix, uplo=_uplo(uplo), diag=_diag(diag))
        return 0, float(_t(Norm.from_string(str(norm)), Am, None, _opts()))
    g["trcon"] = trcon

    # ---- mixed precision (scalapack_gesv_mixed.cc: pdsgesv / pzcgesv)
    if pfx in "dz":
        def gesv_mixed(n, nrhs, a, ia, ja, desca, ipiv, b, ib, jb, descb, x, ix, jx, descx):
            """(info, iter); ipiv 1-based relative to the sub-matrix."""
            from ..models.mixed import gesv_mixed as _g
            A, B, X = _Loc(a, desca, dt), _Loc(b, descb, dt), _Loc(x, descx, dt)
            Am, _ = _sub(A, ia, ja, n, n)
            Bm, _ = _sub(B, ib, jb, n, nrhs)
            Xm, done = _sub(X, ix, jx, n, nrhs)
            piv = Pivots()
            info, it = _g(Am, piv, Bm, Xm, _opts())
            done()
            X.writeback()
            p = (piv.ipiv.cpu() + 1)
            if isinstance(ipiv, np.ndarray):
                ipiv[:p.numel()] = p.numpy()
            else:
                ipiv[:p.numel()] = p.to(ipiv.device, ipiv.dtype)
            return info, it
        g["gesv_mixed"] = gesv_mixed

    # ---- eigenvalues by divide and conquer (scalapack_heevd.cc)
    def heevd(jobz, uplo, n, a, ia, ja, desca, w, z=None, iz=1, jz=1, descz=None):
        return heev(jobz, uplo, n, a, ia, ja, desca, w, z, iz, jz, descz)
    g["heevd" if dt.is_complex else "syevd"] = heevd
    return g


def _install():
    mod = globals()
    for pfx in _PFX:
        for name, fn in _make(pfx).items():
            fn.__name__ = "p" + pfx + name
            mod["p" + pfx + name] = fn


_install()
