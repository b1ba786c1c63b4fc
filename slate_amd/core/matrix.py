"""Distributed matrix types (`include/slate/BaseMatrix.hh`, `Matrix.hh`,
`BaseTrapezoidMatrix.hh`, `TrapezoidMatrix.hh`, `TriangularMatrix.hh`,
`SymmetricMatrix.hh`, `HermitianMatrix.hh`, `BaseBandMatrix.hh`,
`BandMatrix.hh`, `TriangularBandMatrix.hh`, `HermitianBandMatrix.hh`).

Views are cheap: ``sub``/``slice``/``transpose``/``conj_transpose`` only
change offsets and ``op`` and share the :class:`MatrixStorage`.  Typed
views (Triangular, Hermitian, ...) are shallow conversions of each other,
as in SLATE (`HermitianMatrix AH(A)`).

Local-block access (:meth:`BaseMatrix.local_block`) is the MI355X fast
path: for block-cyclic storage it returns the view's local part as ONE
strided tensor of the contiguous local buffer plus the global-index
mapping, so drivers issue one kernel per step instead of one per tile.
"""
from __future__ import annotations

import copy as _copy
from dataclasses import dataclass
from typing import Optional

import torch

from .. import _native
from ..parallel import comm as _comm
from . import func
from .enums import Diag, GridOrder, Layout, Op, Target, TileKind, Uplo
from .exceptions import SlateError, slate_assert
from .storage import DEV, HOST, MatrixStorage, l2g, local_start
from .tile import Tile

HostNum = -1


def _slot_for(device) -> int:
    if device is None:
        return DEV if torch.cuda.is_available() else HOST
    if isinstance(device, int):
        return HOST if device == HostNum else DEV
    if isinstance(device, Target):
        return DEV if device == Target.Devices else HOST
    return DEV if torch.device(device).type == "cuda" else HOST


@dataclass
class LocalBlock:
    """Local part of a (block-cyclic) matrix view."""
    data: torch.Tensor      # (mloc x nloc) strided view, column-major, NOT op'ed
    op: Op                  # logical op of the view
    row_off: int            # local row index of data[0, :] within the rank's local buffer
    col_off: int
    mb: int                 # tile sizes of the distribution
    nb: int
    p: int
    q: int
    pr: int
    pc: int
    grow0: int              # global row of the view's (untransposed) first row
    gcol0: int

    @property
    def mloc(self):
        return self.data.shape[0]

    @property
    def nloc(self):
        return self.data.shape[1]

    def global_row(self, l):
        return l2g(l + self.row_off, self.mb, self.pr, self.p) - self.grow0

    def global_col(self, l):
        return l2g(l + self.col_off, self.nb, self.pc, self.q) - self.gcol0

    def mask(self, mode):
        """TriMask tuple for the kernels: keep global (view-relative) row >= col
        (mode 1) or <= (mode 2)."""
        return (mode, self.mb, self.p, self.pr, self.q, self.pc, self.row_off, self.col_off,
                self.gcol0 - self.grow0)


class BaseMatrix:
    """Shared-storage view (SLATE BaseMatrix)."""

    _kind = "general"

    def __init__(self, storage: MatrixStorage, ioffset=0, joffset=0, mt=None, nt=None,
                 row0_offset=0, col0_offset=0, last_mb=None, last_nb=None,
                 op=Op.NoTrans, uplo=Uplo.General, diag=Diag.NonUnit):
        self.storage = storage
        self.ioffset, self.joffset = ioffset, joffset
        self._mt = storage.mt - ioffset if mt is None else mt
        self._nt = storage.nt - joffset if nt is None else nt
        self.row0_offset, self.col0_offset = row0_offset, col0_offset
        self.last_mb, self.last_nb = last_mb, last_nb
        self._op = Op(op)
        self._uplo = Uplo(uplo)
        self._diag = Diag(diag)

    # ---------------------------------------------------------------- copy
    def _clone(self, cls=None, **kw):
        new = _copy.copy(self)
        if cls is not None:
            new.__class__ = cls
        for k, v in kw.items():
            setattr(new, k, v)
        return new

    # ------------------------------------------------------------ geometry
    def _utile_mb(self, i):   # untransposed
        s = self.storage.tileMb(self.ioffset + i)
        if i == 0:
            s -= self.row0_offset
        if i == self._mt - 1 and self.last_mb is not None:
            s = self.last_mb if self._mt > 1 else min(s, self.last_mb)
        return s

    def _utile_nb(self, j):
        s = self.storage.tileNb(self.joffset + j)
        if j == 0:
            s -= self.col0_offset
        if j == self._nt - 1 and self.last_nb is not None:
            s = self.last_nb if self._nt > 1 else min(s, self.last_nb)
        return s

    def _um(self):
        return sum(self._utile_mb(i) for i in range(self._mt)) if self._mt else 0

    def _un(self):
        return sum(self._utile_nb(j) for j in range(self._nt)) if self._nt else 0

    def mt(self):
        return self._mt if self._op == Op.NoTrans else self._nt

    def nt(self):
        return self._nt if self._op == Op.NoTrans else self._mt

    def m(self):
        return self._um() if self._op == Op.NoTrans else self._un()

    def n(self):
        return self._un() if self._op == Op.NoTrans else self._um()

    def tileMb(self, i):
        return self._utile_mb(i) if self._op == Op.NoTrans else self._utile_nb(i)

    def tileNb(self, j):
        return self._utile_nb(j) if self._op == Op.NoTrans else self._utile_mb(j)

    def op(self):
        return self._op

    def uplo(self):
        """Logical uplo (of op(A)); the stored triangle is uploPhysical()."""
        if self._uplo == Uplo.General or self._op == Op.NoTrans:
            return self._uplo
        return Uplo.Upper if self._uplo == Uplo.Lower else Uplo.Lower

    def diag(self):
        return self._diag

    def uploPhysical(self):
        return self._uplo

    def uploLogical(self):
        return self.uplo()

    @property
    def dtype(self):
        return self.storage.dtype

    @property
    def device(self):
        return self.storage.device

    def comm(self):
        return self.storage.comm

    def mpiRank(self):
        return self.storage.rank

    def gridinfo(self):
        """(order, p, q, myrow, mycol) as SLATE `gridinfo`."""
        bc = self.storage.bc
        if bc is None:
            ok, order, p, q = func.is_2d_cyclic_grid(self.storage.mt, self.storage.nt, self.storage.tileRank)
            if not ok:
                return GridOrder.Unknown, -1, -1, -1, -1
            return order, p, q, -1, -1
        return bc.order, bc.p, bc.q, bc.pr, bc.pc

    # ------------------------------------------------------- tile indexing
    def _global_ij(self, i, j):
        if self._op == Op.NoTrans:
            return self.ioffset + i, self.joffset + j
        return self.ioffset + j, self.joffset + i

    def tileRank(self, i, j):
        return self.storage.tileRank(self._global_ij(i, j))

    def tileDevice(self, i, j):
        return 0

    def tileIsLocal(self, i, j):
        return self.tileRank(i, j) == self.storage.rank

    def tileExists(self, i, j, device=None):
        gi, gj = self._global_ij(i, j)
        return self.storage.tileExists(gi, gj, None if device is None else _slot_for(device))

    def _tile_from_data(self, data, i, j, slot):
        """Apply the view's first-row/col offsets and op to a stored tile."""
        gi, gj = self._global_ij(i, j)
        ui, uj = gi - self.ioffset, gj - self.joffset
        r0 = self.row0_offset if ui == 0 else 0
        c0 = self.col0_offset if uj == 0 else 0
        d = data[r0:r0 + self._utile_mb(ui), c0:c0 + self._utile_nb(uj)]
        uplo = Uplo.General
        if self._uplo != Uplo.General and ui == uj:
            uplo = self.uploPhysical()
            uplo = self._uplo if self._op == Op.NoTrans else (Uplo.Upper if self._uplo == Uplo.Lower else Uplo.Lower)
            uplo = Uplo.Lower if (self.uploPhysical() == Uplo.Lower) else Uplo.Upper
        kind = TileKind.SlateOwned
        t = Tile(d, Op.NoTrans, uplo, kind, slot=slot)
        if self._op == Op.Trans:
            t = t.transpose()
        elif self._op == Op.ConjTrans:
            t = t.conj_transpose()
        return t

    def __call__(self, i, j, device=None) -> Tile:
        """Tile (i, j) in the given memory space (HostNum=-1 or device 0)."""
        slot = self._default_slot() if device is None else _slot_for(device)
        gi, gj = self._global_ij(i, j)
        data = self.storage.tile_data(gi, gj, slot)
        if data is None:
            raise SlateError(f"tile ({i},{j}) has no instance in slot {slot}")
        return self._tile_from_data(data, i, j, slot)

    at = __call__

    def _default_slot(self):
        s = self.storage.origin_slot
        return s if s is not None else _slot_for(None)

    # --------------------------------------------------------------- views
    def sub(self, i1, i2, j1=None, j2=None):
        """Tile-index sub-matrix [i1..i2] x [j1..j2] (inclusive), shared storage."""
        if j1 is None:
            j1, j2 = i1, i2
        if self._op != Op.NoTrans:
            i1, i2, j1, j2 = j1, j2, i1, i2
        mt = max(0, i2 - i1 + 1)
        nt = max(0, j2 - j1 + 1)
        new = self._clone(
            ioffset=self.ioffset + i1, joffset=self.joffset + j1, _mt=mt, _nt=nt,
            row0_offset=self.row0_offset if i1 == 0 else 0,
            col0_offset=self.col0_offset if j1 == 0 else 0,
            last_mb=self.last_mb if (i1 + mt == self._mt) else None,
            last_nb=self.last_nb if (j1 + nt == self._nt) else None)
        return new

    def slice(self, row1, row2, col1, col2):
        """Element-index sub-matrix [row1..row2] x [col1..col2] (inclusive)."""
        if self._op != Op.NoTrans:
            row1, row2, col1, col2 = col1, col2, row1, row2
        s = self.storage
        R0 = s.row_offsets[self.ioffset] + self.row0_offset
        C0 = s.col_offsets[self.joffset] + self.col0_offset
        gr1, gr2, gc1, gc2 = R0 + row1, R0 + row2, C0 + col1, C0 + col2
        i1 = _tile_index(s.row_offsets, gr1)
        i2 = _tile_index(s.row_offsets, gr2)
        j1 = _tile_index(s.col_offsets, gc1)
        j2 = _tile_index(s.col_offsets, gc2)
        new = self._clone(
            ioffset=i1, joffset=j1, _mt=i2 - i1 + 1, _nt=j2 - j1 + 1,
            row0_offset=gr1 - s.row_offsets[i1], col0_offset=gc1 - s.col_offsets[j1],
            last_mb=gr2 - s.row_offsets[i2] + 1, last_nb=gc2 - s.col_offsets[j2] + 1)
        if new._mt == 1:
            new.last_mb = gr2 - gr1 + 1
        if new._nt == 1:
            new.last_nb = gc2 - gc1 + 1
        return new

    def transpose(self):
        if self._op == Op.ConjTrans:
            raise SlateError("transpose of conj-transposed matrix")
        return self._clone(_op=Op.Trans if self._op == Op.NoTrans else Op.NoTrans)

    def conj_transpose(self):
        if self._op == Op.Trans:
            raise SlateError("conj_transpose of transposed matrix")
        return self._clone(_op=Op.ConjTrans if self._op == Op.NoTrans else Op.NoTrans)

    # ------------------------------------------------------------- tiles
    def insertLocalTiles(self, target=Target.Host, device=None):
        """Allocate all local tiles (contiguous local buffer when block-cyclic)."""
        slot = _slot_for(device if device is not None else target)
        s = self.storage
        if s.bc is not None:
            if slot not in s.local:
                s.allocate_local(slot)
            return
        for j in range(self.nt()):
            for i in range(self.mt()):
                if self.tileIsLocal(i, j) and self._in_shape(i, j):
                    gi, gj = self._global_ij(i, j)
                    if not s.tileExists(gi, gj, slot):
                        s.tileInsert(gi, gj, slot)

    def _in_shape(self, i, j):
        return True

    def tileInsert(self, i, j, device=HostNum, data=None):
        gi, gj = self._global_ij(i, j)
        kind = TileKind.UserOwned if data is not None else TileKind.SlateOwned
        d = self.storage.tileInsert(gi, gj, _slot_for(device), data, kind)
        return self._tile_from_data(d, i, j, _slot_for(device))

    def tileInsertWorkspace(self, i, j, device=HostNum):
        gi, gj = self._global_ij(i, j)
        d = self.storage.tileInsert(gi, gj, _slot_for(device), None, TileKind.Workspace, origin=False)
        return self._tile_from_data(d, i, j, _slot_for(device))

    def tileErase(self, i, j, device=None):
        gi, gj = self._global_ij(i, j)
        self.storage.tileErase(gi, gj, None if device is None else _slot_for(device))

    def tileRelease(self, i, j, device=HostNum):
        gi, gj = self._global_ij(i, j)
        self.storage.tileRelease(gi, gj, _slot_for(device))

    def tileGetForReading(self, i, j, device=None, hold=False):
        gi, gj = self._global_ij(i, j)
        slot = _slot_for(device) if device is not None else self._default_slot()
        self.storage.tileGet(gi, gj, slot, modify=False, hold=hold)
        return self(i, j, device if device is not None else (HostNum if slot == HOST else 0))

    def tileGetForWriting(self, i, j, device=None, hold=False):
        gi, gj = self._global_ij(i, j)
        slot = _slot_for(device) if device is not None else self._default_slot()
        self.storage.tileGet(gi, gj, slot, modify=True, hold=hold)
        return self(i, j, device if device is not None else (HostNum if slot == HOST else 0))

    def tileGetAndHold(self, i, j, device=None):
        return self.tileGetForReading(i, j, device, hold=True)

    def tileGetAllForReading(self, device=None):
        for j in range(self.nt()):
            for i in range(self.mt()):
                if self.tileIsLocal(i, j) and self._in_shape(i, j):
                    self.tileGetForReading(i, j, device)

    def tileGetAllForWriting(self, device=None):
        for j in range(self.nt()):
            for i in range(self.mt()):
                if self.tileIsLocal(i, j) and self._in_shape(i, j):
                    self.tileGetForWriting(i, j, device)

    def tileModified(self, i, j, device=None, permissive=False):
        gi, gj = self._global_ij(i, j)
        slot = _slot_for(device) if device is not None else self._default_slot()
        self.storage.tileModified(gi, gj, slot, permissive)

    def tileState(self, i, j, device=None):
        gi, gj = self._global_ij(i, j)
        slot = _slot_for(device) if device is not None else self._default_slot()
        return self.storage.tileState(gi, gj, slot)

    def tileOnHold(self, i, j, device=None):
        return bool(self.tileState(i, j, device) & 0x1000)

    def tileUnsetHold(self, i, j, device=None):
        gi, gj = self._global_ij(i, j)
        slot = _slot_for(device) if device is not None else self._default_slot()
        self.storage.table.unhold(gi, gj, slot)

    def tileUpdateOrigin(self, i, j):
        gi, gj = self._global_ij(i, j)
        self.storage.tileUpdateOrigin(gi, gj)

    def tileUpdateAllOrigin(self):
        self.storage.sync_origin()

    def releaseWorkspace(self):
        self.storage.releaseWorkspace()

    def clearWorkspace(self):
        self.storage.clearWorkspace()

    def releaseLocalWorkspace(self):
        self.storage.clearWorkspace()

    def releaseRemoteWorkspace(self):
        self.storage.clearWorkspace()

    def tileLayout(self, i, j):
        return Layout.ColMajor

    # --------------------------------------------------------- fast path
    def is_block_cyclic(self):
        return self.storage.bc is not None and bool(self.storage.local)

    def local_block(self, slot=None) -> LocalBlock:
        """Local part of this view as one strided tensor (block-cyclic only).
        The data is returned un-op'ed; ``op`` tells the caller how to read it."""
        s = self.storage
        bc = s.bc
        slate_assert(bc is not None, "local_block requires block-cyclic storage")
        if slot is None:
            slot = s.origin_slot if s.origin_slot is not None else _slot_for(None)
        buf = s.prepare_local(slot)
        R0 = s.row_offsets[self.ioffset] + self.row0_offset
        C0 = s.col_offsets[self.joffset] + self.col0_offset
        R1, C1 = R0 + self._um(), C0 + self._un()
        if bc.pr < 0:
            data = buf[0:0, 0:0]
            return LocalBlock(data, self._op, 0, 0, bc.mb, bc.nb, bc.p, bc.q, 0, 0, R0, C0)
        lr0, lr1 = local_start(R0, bc.mb, bc.pr, bc.p), local_start(R1, bc.mb, bc.pr, bc.p)
        lc0, lc1 = local_start(C0, bc.nb, bc.pc, bc.q), local_start(C1, bc.nb, bc.pc, bc.q)
        return LocalBlock(buf[lr0:lr1, lc0:lc1], self._op, lr0, lc0, bc.mb, bc.nb, bc.p, bc.q,
                          bc.pr, bc.pc, R0, C0)

    def global_offsets(self):
        """(first global row, first global col) of the untransposed view."""
        s = self.storage
        return s.row_offsets[self.ioffset] + self.row0_offset, s.col_offsets[self.joffset] + self.col0_offset

    # --------------------------------------------------------- constructors
    def emptyLike(self, mb=None, nb=None, op=Op.NoTrans, dtype=None):
        """New matrix with the same distribution (no tiles allocated)."""
        s = self.storage
        bc = s.bc
        if op != Op.NoTrans:
            base = self.transpose() if op == Op.Trans else self.conj_transpose()
            m, n = base.m(), base.n()
        else:
            m, n = self.m(), self.n()
        dtype = dtype or s.dtype
        if bc is not None and mb is None and nb is None and self.ioffset == 0 and self.joffset == 0 \
                and self.row0_offset == 0 and self.col0_offset == 0:
            if op == Op.NoTrans:
                st = MatrixStorage(m, n, func.uniform_blocksize(m, bc.mb), func.uniform_blocksize(n, bc.nb),
                                   func.process_2d_grid(bc.order, bc.p, bc.q), s.comm, dtype, s.device)
            else:
                st = MatrixStorage(m, n, func.uniform_blocksize(m, bc.nb), func.uniform_blocksize(n, bc.mb),
                                   func.transpose_grid(func.process_2d_grid(bc.order, bc.p, bc.q)),
                                   s.comm, dtype, s.device)
        else:
            # same tile ownership as this view (tile-index aligned)
            view = self if op == Op.NoTrans else (self.transpose() if op == Op.Trans else self.conj_transpose())
            mt, nt = view.mt(), view.nt()
            tmb = [view.tileMb(i) if mb is None else mb for i in range(mt)]
            tnb = [view.tileNb(j) if nb is None else nb for j in range(nt)]
            m2, n2 = sum(tmb), sum(tnb)
            rk = view.tileRank
            def fmb(i, _t=tmb): return _t[i] if i < len(_t) else _t[-1]
            def fnb(j, _t=tnb): return _t[j] if j < len(_t) else _t[-1]
            if mb is None and nb is None and bc is not None and self.row0_offset == 0 and self.col0_offset == 0 \
                    and op == Op.NoTrans and all(x == tmb[0] for x in tmb[:-1]) and all(x == tnb[0] for x in tnb[:-1]):
                io, jo = self.ioffset, self.joffset
                def rank(ij, _io=io, _jo=jo, _r=s.tileRank): return _r((ij[0] + _io, ij[1] + _jo))
                fmb = func.uniform_blocksize(m2, tmb[0]) if tmb else fmb
                fnb = func.uniform_blocksize(n2, tnb[0]) if tnb else fnb
                # a shifted block-cyclic grid is still 2D cyclic
                st = MatrixStorage(m2, n2, fmb, fnb, rank, s.comm, dtype, s.device)
            else:
                st = MatrixStorage(m2, n2, fmb, fnb, lambda ij, _v=view: _v.tileRank(ij[0], ij[1]),
                                   s.comm, dtype, s.device)
        return self._new_of_kind(st)

    def _new_of_kind(self, st):
        return Matrix(_storage=st)

    def __repr__(self):
        return (f"{type(self).__name__}({self.m()}x{self.n()}, tiles {self.mt()}x{self.nt()}, "
                f"op={self._op.name}, uplo={self._uplo.name}, dtype={self.dtype}, "
                f"rank={self.storage.rank}/{self.storage.comm.size})")


def _tile_index(offsets, g):
    lo, hi = 0, len(offsets) - 2
    while lo < hi:
        mid = (lo + hi + 1) // 2
        if offsets[mid] <= g:
            lo = mid
        else:
            hi = mid - 1
    return lo


def _make_storage(m, n, mb, nb, p, q, comm, dtype, device, order=GridOrder.Col):
    comm = comm or _comm.world()
    if p is None or q is None:
        p, q = (1, 1) if comm.size == 1 else func.grid_shape(comm.size)
    return MatrixStorage(m, n, func.uniform_blocksize(m, mb), func.uniform_blocksize(n, nb),
                         func.process_2d_grid(order, p, q), comm, dtype, device)


class Matrix(BaseMatrix):
    """General m x n distributed matrix (`include/slate/Matrix.hh`)."""

    def __init__(self, m=0, n=0, nb=256, p=None, q=None, comm=None, dtype=torch.float64,
                 device=None, mb=None, order=GridOrder.Col, _storage=None, **kw):
        if _storage is None:
            _storage = _make_storage(m, n, mb or nb, nb, p, q, comm, dtype, device, GridOrder.from_string(order))
        super().__init__(_storage, **kw)

    @classmethod
    def from_functions(cls, m, n, tileMb, tileNb, tileRank, tileDevice=None, comm=None,
                       dtype=torch.float64, device=None):
        """Lambda constructor (BaseMatrix.hh:855-931)."""
        st = MatrixStorage(m, n, tileMb, tileNb, tileRank, comm or _comm.world(), dtype, device, tileDevice)
        return cls(_storage=st)

    @classmethod
    def fromLAPACK(cls, m, n, A: torch.Tensor, lda=None, mb=None, nb=None, p=1, q=1, comm=None):
        """Wrap an lda x n column-major array replicated on every rank."""
        return cls._from_lapack(cls, m, n, A, lda, mb, nb, p, q, comm)

    @staticmethod
    def _from_lapack(kls, m, n, A, lda, mb, nb, p, q, comm, **kw):
        comm = comm or _comm.world()
        nb = nb or 256
        mb = mb or nb
        A2 = _as_colmajor(A, m, n, lda)
        st = MatrixStorage(m, n, func.uniform_blocksize(m, mb), func.uniform_blocksize(n, nb),
                           func.process_2d_grid(GridOrder.Col, p, q), comm, A2.dtype, A2.device)
        slot = _slot_for(A2.device)
        if p * q == 1:
            st.allocate_local(slot, A2, TileKind.UserOwned)
        else:
            st.bc = None
            for j in range(st.nt):
                for i in range(st.mt):
                    if st.tileIsLocal(i, j):
                        r0, c0 = st.row_offsets[i], st.col_offsets[j]
                        st.tileInsert(i, j, slot, A2[r0:r0 + st.tileMb(i), c0:c0 + st.tileNb(j)],
                                      TileKind.UserOwned)
        return kls(_storage=st, **kw)

    @classmethod
    def fromScaLAPACK(cls, m, n, A: torch.Tensor, lld=None, mb=None, nb=None, order=GridOrder.Col,
                      p=1, q=1, comm=None):
        """Wrap this rank's ScaLAPACK local array (lld x nloc, column-major)."""
        return cls._from_scalapack(cls, m, n, A, lld, mb, nb, order, p, q, comm)

    @staticmethod
    def _from_scalapack(kls, m, n, A, lld, mb, nb, order, p, q, comm, **kw):
        comm = comm or _comm.world()
        nb = nb or 256
        mb = mb or nb
        st = MatrixStorage(m, n, func.uniform_blocksize(m, mb), func.uniform_blocksize(n, nb),
                           func.process_2d_grid(GridOrder.from_string(order), p, q), comm, A.dtype, A.device)
        bc = st.bc
        A2 = _as_colmajor(A, max(bc.mloc, 1) if A.dim() == 1 else A.shape[0], bc.nloc, lld)
        st.allocate_local(_slot_for(A2.device), A2, TileKind.UserOwned)
        return kls(_storage=st, **kw)

    @classmethod
    def fromDevices(cls, m, n, Aarray, lda=None, mb=None, nb=None, p=1, q=1, comm=None):
        """Wrap device-resident local arrays (one per device; one device per rank)."""
        A = Aarray[0] if isinstance(Aarray, (list, tuple)) else Aarray
        return cls.fromScaLAPACK(m, n, A, lda, mb, nb, GridOrder.Col, p, q, comm)

    # ---- utilities -------------------------------------------------------
    def gather(self, root=0) -> Optional[torch.Tensor]:
        """Assemble the full matrix on `root` (returns None elsewhere)."""
        from ..models.aux import gather
        return gather(self, root)

    def to_dense(self) -> torch.Tensor:
        """Full matrix replicated on every rank (testing / small problems)."""
        from ..models.aux import allgather_dense
        return allgather_dense(self)

    def getMaxHostTiles(self):
        return sum(1 for j in range(self.nt()) for i in range(self.mt()) if self.tileIsLocal(i, j))

    getMaxDeviceTiles = getMaxHostTiles

    def allocateBatchArrays(self, batch_size=0, num_arrays=1):
        """Pointer arrays are built on demand by the grouped kernels; kept for API parity."""
        return None

    def reserveDeviceWorkspace(self):
        return None

    def reserveHostWorkspace(self):
        return None


def _as_colmajor(A, m, n, ld):
    """View a user array as an m x n column-major matrix (lda >= m)."""
    if A.dim() == 1:
        ld = ld or m
        return A.as_strided((m, n), (1, ld))
    if A.stride(0) == 1 or A.shape[0] <= 1:
        if ld is not None and ld != A.stride(1) and A.shape[1] > 1:
            return A.as_strided((m, n), (1, ld))
        return A[:m, :n]
    raise SlateError("array must be column-major (stride(0) == 1); pass A.t().contiguous().t()")


class BaseTrapezoidMatrix(BaseMatrix):
    _kind = "trapezoid"

    def _in_shape(self, i, j):
        gi, gj = self._global_ij(i, j)
        if self.storage.bc is not None:
            return True
        return gi >= gj if self.uploPhysical() == Uplo.Lower else gi <= gj

    def _new_of_kind(self, st):
        return type(self)(self._uplo, _storage=st, diag=self._diag) if isinstance(self, TriangularMatrix) \
            else type(self)(self._uplo, _storage=st)


class TrapezoidMatrix(BaseTrapezoidMatrix):
    def __init__(self, uplo=Uplo.Lower, m=0, n=0, nb=256, p=None, q=None, comm=None, dtype=torch.float64,
                 device=None, diag=Diag.NonUnit, _storage=None, matrix: Optional[BaseMatrix] = None, **kw):
        if matrix is not None:
            self.__dict__.update(matrix.__dict__)
            self._uplo, self._diag = Uplo(uplo), Diag(diag)
            return
        if _storage is None:
            _storage = _make_storage(m, n, nb, nb, p, q, comm, dtype, device)
        super().__init__(_storage, uplo=uplo, diag=diag, **kw)

    @classmethod
    def fromLAPACK(cls, uplo, m, n, A, lda=None, nb=None, p=1, q=1, comm=None, diag=Diag.NonUnit):
        M = Matrix._from_lapack(Matrix, m, n, A, lda, nb, nb, p, q, comm)
        return cls(uplo, matrix=M, diag=diag)

    @classmethod
    def fromScaLAPACK(cls, uplo, m, n, A, lld=None, nb=None, p=1, q=1, comm=None, diag=Diag.NonUnit,
                      order=GridOrder.Col):
        M = Matrix._from_scalapack(Matrix, m, n, A, lld, nb, nb, order, p, q, comm)
        return cls(uplo, matrix=M, diag=diag)


class TriangularMatrix(TrapezoidMatrix):
    """Square triangular matrix with Diag (`TriangularMatrix.hh`)."""

    def __init__(self, uplo=Uplo.Lower, n_or_diag=None, *args, diag=Diag.NonUnit, matrix=None, **kw):
        if isinstance(n_or_diag, (Diag, str)) and not isinstance(n_or_diag, int):
            diag = Diag(n_or_diag)
            n_or_diag = None
            if args and isinstance(args[0], BaseMatrix):      # (uplo, diag, A)
                matrix, args = args[0], args[1:]
            elif args:                                         # (uplo, diag, n, ...)
                n_or_diag, args = args[0], args[1:]
        if matrix is not None:
            TrapezoidMatrix.__init__(self, uplo, matrix=matrix, diag=diag)
            return
        if isinstance(n_or_diag, BaseMatrix):
            TrapezoidMatrix.__init__(self, uplo, matrix=n_or_diag, diag=diag)
            return
        n = n_or_diag or 0
        TrapezoidMatrix.__init__(self, uplo, n, n, *args, diag=diag, **kw)

    @classmethod
    def fromLAPACK(cls, uplo, diag, n, A, lda=None, nb=None, p=1, q=1, comm=None):
        M = Matrix._from_lapack(Matrix, n, n, A, lda, nb, nb, p, q, comm)
        return cls(uplo, matrix=M, diag=diag)

    @classmethod
    def fromScaLAPACK(cls, uplo, diag, n, A, lld=None, nb=None, p=1, q=1, comm=None, order=GridOrder.Col):
        M = Matrix._from_scalapack(Matrix, n, n, A, lld, nb, nb, order, p, q, comm)
        return cls(uplo, matrix=M, diag=diag)


class _SquareSym(BaseTrapezoidMatrix):
    def __init__(self, uplo=Uplo.Lower, n=0, nb=256, p=None, q=None, comm=None, dtype=torch.float64,
                 device=None, _storage=None, matrix: Optional[BaseMatrix] = None, **kw):
        if isinstance(n, BaseMatrix):
            matrix, n = n, 0
        if matrix is not None:
            self.__dict__.update(matrix.__dict__)
            self._uplo = Uplo(uplo)
            self._diag = Diag.NonUnit
            return
        if _storage is None:
            _storage = _make_storage(n, n, nb, nb, p, q, comm, dtype, device)
        super().__init__(_storage, uplo=uplo, **kw)

    def _new_of_kind(self, st):
        return type(self)(self._uplo, _storage=st)

    @classmethod
    def fromLAPACK(cls, uplo, n, A, lda=None, nb=None, p=1, q=1, comm=None):
        M = Matrix._from_lapack(Matrix, n, n, A, lda, nb, nb, p, q, comm)
        return cls(uplo, matrix=M)

    @classmethod
    def fromScaLAPACK(cls, uplo, n, A, lld=None, nb=None, p=1, q=1, comm=None, order=GridOrder.Col):
        M = Matrix._from_scalapack(Matrix, n, n, A, lld, nb, nb, order, p, q, comm)
        return cls(uplo, matrix=M)


class SymmetricMatrix(_SquareSym):
    _kind = "symmetric"


class HermitianMatrix(_SquareSym):
    _kind = "hermitian"


# ------------------------------------------------------------------ band
def _band_storage(m, n, nb, kl_store, ku_store, comm, dtype, device):
    """Compact band storage (core/band_storage.py): only the tiles within
    kl_store / ku_store of the diagonal exist, 1-D column-cyclic over all
    ranks (the p x q arguments of the band constructors only fix the
    communicator, as ScaLAPACK's band routines use a 1-D grid)."""
    from .band_storage import BandStorage, tiles_for
    comm = comm or _comm.world()
    return BandStorage(m, n, nb, tiles_for(kl_store, nb), tiles_for(ku_store, nb), comm, dtype, device)


class BaseBandMatrix(BaseMatrix):
    """Band matrix: kl sub-, ku super-diagonals (`BaseBandMatrix.hh:27-368`).

    Compact storage: only the tiles touching the band (plus, for general
    band matrices, the kl extra upper tile diagonals of the LU fill-in) are
    allocated, as per-column slabs (core/band_storage.py)."""

    def __init__(self, storage, kl, ku, **kw):
        super().__init__(storage, **kw)
        self._kl, self._ku = kl, ku

    def lowerBandwidth(self):
        return self._kl if self._op == Op.NoTrans else self._ku

    def upperBandwidth(self):
        return self._ku if self._op == Op.NoTrans else self._kl

    def setLowerBandwidth(self, kl):
        self._kl = kl

    def setUpperBandwidth(self, ku):
        self._ku = ku

    def _in_shape(self, i, j):
        s = self.storage
        gi, gj = self._global_ij(i, j)
        r0, r1 = s.row_offsets[gi], s.row_offsets[gi + 1] - 1
        c0, c1 = s.col_offsets[gj], s.col_offsets[gj + 1] - 1
        # tile intersects band: exists (r, c) with -ku <= r - c <= kl
        return (r1 - c0 >= -self._ku) and (r0 - c1 <= self._kl)


class BandMatrix(BaseBandMatrix):
    def __init__(self, m=0, n=0, kl=0, ku=0, nb=256, p=None, q=None, comm=None, dtype=torch.float64,
                 device=None, _storage=None, matrix=None, **kw):
        if matrix is not None:
            self.__dict__.update(matrix.__dict__)
            self._kl, self._ku = kl, ku
            return
        if _storage is None:
            _storage = _band_storage(m, n, nb, kl, ku + kl, comm, dtype, device)
        super().__init__(_storage, kl, ku, **kw)

    def _new_of_kind(self, st):
        return BandMatrix(kl=self._kl, ku=self._ku, _storage=st)


class BaseTriangularBandMatrix(BaseBandMatrix):
    def __init__(self, storage, uplo, kd, **kw):
        kl, ku = (kd, 0) if Uplo(uplo) == Uplo.Lower else (0, kd)
        super().__init__(storage, kl, ku, uplo=uplo, **kw)
        self._kd = kd

    def bandwidth(self):
        return self._kd


class TriangularBandMatrix(BaseTriangularBandMatrix):
    _kind = "trapezoid"

    def __init__(self, uplo=Uplo.Lower, diag=Diag.NonUnit, n=0, kd=0, nb=256, p=None, q=None, comm=None,
                 dtype=torch.float64, device=None, _storage=None, matrix=None, **kw):
        if matrix is not None:
            self.__dict__.update(matrix.__dict__)
            self._uplo, self._diag, self._kd = Uplo(uplo), Diag(diag), kd
            self._kl, self._ku = (kd, 0) if self._uplo == Uplo.Lower else (0, kd)
            return
        if _storage is None:
            lo = Uplo(uplo) == Uplo.Lower
            _storage = _band_storage(n, n, nb, kd if lo else 0, 0 if lo else kd, comm, dtype, device)
        super().__init__(_storage, uplo, kd, diag=diag, **kw)


class HermitianBandMatrix(BaseTriangularBandMatrix):
    _kind = "hermitian"

    def __init__(self, uplo=Uplo.Lower, n=0, kd=0, nb=256, p=None, q=None, comm=None, dtype=torch.float64,
                 device=None, _storage=None, matrix=None, **kw):
        if matrix is not None:
            self.__dict__.update(matrix.__dict__)
            self._uplo, self._kd = Uplo(uplo), kd
            self._kl, self._ku = (kd, 0) if self._uplo == Uplo.Lower else (0, kd)
            return
        if _storage is None:
            lo = Uplo(uplo) == Uplo.Lower
            _storage = _band_storage(n, n, nb, kd if lo else 0, 0 if lo else kd, comm, dtype, device)
        super().__init__(_storage, uplo, kd, **kw)


# SLATE's TriangularFactors (geqrf/gelqf/he2hb T), Pivots
class TriangularFactors(list):
    """[Tlocal, Treduce] (`include/slate/slate.hh:856-857`); here the block
    reflector factors are stored per panel in a single matrix-like list."""


class Pivot:
    """SLATE Pivot{tile_index, element_offset} (`include/slate/types.hh:84-117`)."""
    __slots__ = ("tile_index", "element_offset")

    def __init__(self, tile_index, element_offset):
        self.tile_index, self.element_offset = tile_index, element_offset

    def __eq__(self, o):
        return (self.tile_index, self.element_offset) == (o.tile_index, o.element_offset)

    def __repr__(self):
        return f"Pivot({self.tile_index},{self.element_offset})"


class Pivots:
    """Row-pivot vector of a factorization: global 0-based pivot rows, one
    entry per eliminated row (kept as a host int64 tensor plus the device
    mirror used by the row-swap kernels).  ``pivots[k]`` returns the list of
    SLATE-style Pivot records of panel k."""

    def __init__(self, nb=256):
        self._host = torch.zeros(0, dtype=torch.int64)
        self.nb = nb
        self._dev = None

    def set(self, ipiv: torch.Tensor, nb):
        """Store the pivots where they were produced (a factorization leaves
        them on the GPU: no host copy until someone reads ``ipiv``)."""
        ipiv = ipiv.to(torch.int64)
        self.nb = nb
        if ipiv.is_cuda:
            self._dev, self._host = ipiv, None
        else:
            self._dev, self._host = None, ipiv

    @property
    def ipiv(self) -> torch.Tensor:
        if self._host is None:
            self._host = self._dev.cpu()
        return self._host

    @ipiv.setter
    def ipiv(self, v):
        self.set(torch.as_tensor(v, dtype=torch.int64), self.nb)

    def device(self, dev):
        dev = torch.device(dev)
        if self._dev is None or self._dev.device != dev:
            src = self._dev if self._dev is not None else self._host
            self._dev = src.to(dev, non_blocking=src.device.type == "cpu" and src.is_pinned())
        return self._dev

    def __len__(self):
        n = self.size
        return -(-n // self.nb) if n else 0

    @property
    def size(self) -> int:
        """Number of pivots (no host copy)."""
        return (self._dev if self._host is None else self._host).numel()

    def __getitem__(self, k):
        seg = self.ipiv[k * self.nb:(k + 1) * self.nb].tolist()
        return [Pivot(p // self.nb, p % self.nb) for p in seg]
