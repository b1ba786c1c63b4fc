"""Tile: a non-owning view of one mb x nb block (`include/slate/Tile.hh:105-400`).

A tile wraps a 2-D torch tensor *view* in column-major layout (stride(0)
== 1, stride(1) == ld) living in host memory or on this rank's MI355X,
plus the logical attributes SLATE keeps per tile: ``op`` (NoTrans / Trans /
ConjTrans), ``uplo``, ``kind`` (Workspace / SlateOwned / UserOwned) and
``layout``.  Element access and ``mb()/nb()`` honour ``op`` exactly like
SLATE tiles.  Data movement (copy between memory spaces, layout
conversion) goes through :mod:`slate_amd.ops` so it runs on the gfx950
kernels when the data is on the GPU.
"""
from __future__ import annotations

import torch

from .enums import Layout, Op, TileKind, Uplo


class Tile:
    __slots__ = ("_data", "op", "uplo", "kind", "layout", "slot")

    def __init__(self, data: torch.Tensor, op=Op.NoTrans, uplo=Uplo.General,
                 kind=TileKind.SlateOwned, layout=Layout.ColMajor, slot=None):
        if data.dim() != 2:
            raise ValueError("tile data must be 2-D")
        self._data = data
        self.op = Op(op)
        self.uplo = Uplo(uplo)
        self.kind = TileKind(kind)
        self.layout = Layout(layout)
        self.slot = slot if slot is not None else (1 if data.is_cuda else 0)

    # -- geometry (op-aware) ---------------------------------------------
    def mb(self):
        return self._data.shape[0] if self.op == Op.NoTrans else self._data.shape[1]

    def nb(self):
        return self._data.shape[1] if self.op == Op.NoTrans else self._data.shape[0]

    def stride(self):
        return max(1, self._data.stride(1)) if self.layout == Layout.ColMajor else max(1, self._data.stride(0))

    @property
    def data(self) -> torch.Tensor:
        """Underlying stored (un-op'ed) block, column-major view."""
        return self._data

    def tensor(self) -> torch.Tensor:
        """Logical op(tile) as a tensor view."""
        if self.op == Op.NoTrans:
            return self._data
        if self.op == Op.Trans:
            return self._data.mT
        return self._data.mT.conj()

    @property
    def device(self):
        return self._data.device

    def origin(self):
        return self.kind != TileKind.Workspace

    def allocated(self):
        return self.kind != TileKind.UserOwned

    # -- element access ---------------------------------------------------
    def __getitem__(self, ij):
        i, j = ij
        if self.op == Op.NoTrans:
            return self._data[i, j].item()
        v = self._data[j, i].item()
        return v.conjugate() if (self.op == Op.ConjTrans and isinstance(v, complex)) else v

    def at(self, i, j):
        return self[i, j]

    def __setitem__(self, ij, v):
        i, j = ij
        if self.op == Op.NoTrans:
            self._data[i, j] = v
        else:
            self._data[j, i] = v.conjugate() if (self.op == Op.ConjTrans and isinstance(v, complex)) else v

    # -- views --------------------------------------------------------------
    def slice(self, row1, row2, col1, col2):
        """Inclusive sub-block [row1..row2] x [col1..col2] in op coordinates."""
        if self.op == Op.NoTrans:
            d = self._data[row1:row2 + 1, col1:col2 + 1]
        else:
            d = self._data[col1:col2 + 1, row1:row2 + 1]
        return Tile(d, self.op, self.uplo, self.kind, self.layout, self.slot)

    def transpose(self):
        op = Op.Trans if self.op == Op.NoTrans else Op.NoTrans
        if self.op == Op.ConjTrans:
            raise ValueError("transpose of conj-transposed tile is not supported")
        return Tile(self._data, op, self.uplo, self.kind, self.layout, self.slot)

    def conj_transpose(self):
        op = Op.ConjTrans if self.op == Op.NoTrans else Op.NoTrans
        if self.op == Op.Trans:
            raise ValueError("conj_transpose of transposed tile is not supported")
        return Tile(self._data, op, self.uplo, self.kind, self.layout, self.slot)

    def uploPhysical(self):
        if self.uplo == Uplo.General or self.op == Op.NoTrans:
            return self.uplo
        return Uplo.Upper if self.uplo == Uplo.Lower else Uplo.Lower

    def uploLogical(self):
        return self.uplo

    def copyData(self, dst: "Tile"):
        """Copy data into dst (any memory space), honouring neither op."""
        dst._data.copy_(self._data, non_blocking=True)

    def set(self, offdiag, diag=None):
        from .. import ops
        ops.geset(self._data, offdiag, offdiag if diag is None else diag,
                  uplo=self.uplo if self.uplo != Uplo.General else Uplo.General)

    def __repr__(self):
        return (f"Tile({self.mb()}x{self.nb()}, op={self.op.name}, uplo={self.uplo.name}, "
                f"kind={self.kind.name}, device={self.device})")
