"""Compact band storage (SLATE `BaseBandMatrix.hh:27-368`: only the tiles
inside the band exist).

MI355X layout: the tile columns are distributed 1-D block-cyclically over
all ranks (ScaLAPACK's band solvers pdgbtrf/pdpbtrf distribute band
matrices the same way); on each rank the tiles of local tile column j --
tile rows j-KU .. j+KL -- are stacked in ONE column-major slab
(``H nb`` rows, H = KU + KL + 1, leading dimension padded to 16).  A tile is
a strided view into the slab, so the per-tile infrastructure (MOSI table,
tile get/insert, generation, dense conversion for tests) works unchanged,
while the band drivers (models/band.py) see every panel and every
trailing-column update as ONE contiguous sub-block of a slab: memory is
O(n (kl + ku)) per matrix, not O(n^2).

For a general band matrix KU covers the LU fill-in (ku + kl upper
diagonals, `src/gbtrf.cc`: the upper bandwidth grows to kl + ku).
"""
from __future__ import annotations

import torch

from . import func
from .enums import TileKind
from .storage import DEV, MatrixStorage, numroc


def tiles_for(width: int, nb: int) -> int:
    """Tile rows a bandwidth spans beyond the diagonal tile."""
    return -(-max(0, int(width)) // nb) if width > 0 else 0


class BandStorage(MatrixStorage):
    def __init__(self, m, n, nb, KL, KU, comm, dtype=torch.float64, device=None):
        Q = comm.size
        super().__init__(m, n, func.uniform_blocksize(m, nb), func.uniform_blocksize(n, nb),
                         lambda ij: ij[1] % Q, comm, dtype, device)
        self.band_nb = nb
        self.KL, self.KU, self.Q = int(KL), int(KU), Q
        self.H = self.KL + self.KU + 1
        self.slab = {}

    def _detect_block_cyclic(self):
        return None                 # per-tile mode for the generic code paths

    # ---- geometry ------------------------------------------------------
    @property
    def nloc(self):
        return numroc(self.n, self.band_nb, self.rank, self.Q) if self.rank < self.Q else 0

    def window(self, j):
        """Tile rows [lo, hi] stored for tile column j."""
        return max(0, j - self.KU), min(self.mt - 1, j + self.KL)

    def in_window(self, i, j):
        lo, hi = self.window(j)
        return lo <= i <= hi

    def slab_row(self, g, j):
        """Slab row of global row g in tile column j."""
        return g - (j - self.KU) * self.band_nb

    def local_col(self, j):
        return (j // self.Q) * self.band_nb

    def my_cols(self, lo=0, hi=None):
        """Local tile columns j in [lo, hi] (inclusive), ascending."""
        hi = self.nt - 1 if hi is None else min(hi, self.nt - 1)
        lo = max(lo, 0)
        if self.rank >= self.Q or lo > hi:
            return []
        first = lo + ((self.rank - lo) % self.Q)
        return list(range(first, hi + 1, self.Q))

    def get_slab(self, slot):
        buf = self.slab.get(slot)
        if buf is None:
            rows = self.H * self.band_nb
            ld = max(16, -(-rows // 16) * 16)
            buf = torch.zeros((max(self.nloc, 1), ld), dtype=self.dtype, device=self.device_of(slot)).t()[:rows]
            self.slab[slot] = buf
        return buf

    def _alloc_tile(self, i, j, slot, kind):
        if kind == TileKind.Workspace or not self.tileIsLocal(i, j) or not self.in_window(i, j):
            return super()._alloc_tile(i, j, slot, kind)
        buf = self.get_slab(slot)
        r = self.slab_row(self.row_offsets[i], j)
        c = self.local_col(j)
        return buf[r:r + self.tileMb(i), c:c + self.tileNb(j)]

    def band_slot(self):
        """Slot holding the band data (origin), creating the slab if needed."""
        slot = self.origin_slot if self.origin_slot is not None else (DEV if self.device.type == "cuda" else 0)
        self.get_slab(slot)
        return slot

    def sync_slab(self, slot):
        """Make every local tile's latest instance live in the slab of
        ``slot`` (tiles updated elsewhere are copied back)."""
        self.sync_origin()
        return self.get_slab(slot)

    def mark_slab_modified(self, slot):
        self.mark_local_modified(slot)
