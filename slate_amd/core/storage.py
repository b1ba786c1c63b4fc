"""MatrixStorage: the tile map shared by every view of a matrix.

Reference contract: `include/slate/internal/MatrixStorage.hh:151-1152`
(tile map, tileMb/Nb/Rank lambdas, tileInsert/erase/release, workspace,
receive counts) and SURVEY Appendix A (MOSI semantics).

MI355X-first layout decisions
-----------------------------
* One process drives one GPU, so a tile has at most two instances:
  slot ``HOST`` (0) and slot ``DEV`` (1).  Their MOSI states live in the
  native :class:`_host.TileTable` (C++, mutex-protected).
* When the distribution is 2D block-cyclic with uniform tile sizes (the
  default constructor, ``fromScaLAPACK``, ``fromLAPACK``), the local tiles
  are *views into one contiguous column-major local buffer* (ScaLAPACK
  layout, leading dimension padded to 16 elements for 16-byte vector
  loads).  Because block-cyclic ownership preserves tile order, every
  sub-matrix view's local part is a contiguous sub-block of that buffer:
  a whole trailing update becomes ONE MFMA GEMM launch over the local
  buffer (with a triangular mask evaluated in global coordinates), instead
  of SLATE's per-tile batched-BLAS device regions.
* Other distributions (lambdas, non-uniform tiles, band storage) keep
  per-tile tensors; workspace (received remote tiles) comes from a
  per-storage slab pool: on the GPU the native stream-ordered
  :class:`_hip.DevicePool` (hipMalloc'd chunks under an HBM cap, event-
  ordered frees, csrc/hip/devpool.hip); on the host :class:`_host.SlabPool`
  bookkeeping over torch chunks.
"""
from __future__ import annotations

import threading
from dataclasses import dataclass
from typing import Callable, Optional

import torch

from .. import _native
from .enums import GridOrder, Layout, TileKind
from .exceptions import SlateError, slate_assert
from . import func

HOST, DEV = 0, 1
_host = _native._host


def numroc(n: int, nb: int, iproc: int, nprocs: int) -> int:
    """Rows of an n-row block-cyclic dimension owned by iproc (ScaLAPACK numroc)."""
    if n <= 0:
        return 0
    nblocks = n // nb
    num = (nblocks // nprocs) * nb
    extra = nblocks % nprocs
    if iproc < extra:
        num += nb
    elif iproc == extra:
        num += n % nb
    return num


def local_start(g: int, nb: int, iproc: int, nprocs: int) -> int:
    """Number of local indices (owned by iproc) with global index < g."""
    t, r = divmod(g, nb)
    # full tiles before tile t owned by iproc
    cnt = (t - iproc + nprocs - 1) // nprocs if t > iproc else 0
    loc = cnt * nb
    if t % nprocs == iproc:
        loc += r
    return loc


def l2g(l: int, nb: int, iproc: int, nprocs: int) -> int:
    lt, r = divmod(l, nb)
    return (lt * nprocs + iproc) * nb + r


@dataclass
class BlockCyclic:
    mb: int
    nb: int
    p: int
    q: int
    order: GridOrder
    pr: int       # this rank's process row (-1 if not in grid)
    pc: int
    mloc: int
    nloc: int
    lld: int

    def rank_of(self, i, j):
        if self.order == GridOrder.Col:
            return (i % self.p) + (j % self.q) * self.p
        return (i % self.p) * self.q + (j % self.q)


class MatrixStorage:
    def __init__(self, m: int, n: int, tileMb: Callable, tileNb: Callable,
                 tileRank: Callable, comm, dtype=torch.float64,
                 device: Optional[torch.device] = None, tileDevice: Optional[Callable] = None):
        self.m, self.n = int(m), int(n)
        self.tileMb, self.tileNb, self.tileRank = tileMb, tileNb, tileRank
        self.tileDevice = tileDevice or (lambda ij: 0)
        self.comm = comm
        self.rank = comm.rank
        self.dtype = dtype
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
                else torch.device("cpu")
        self.device = torch.device(device)
        self.mt = self._count_tiles(self.m, tileMb)
        self.nt = self._count_tiles(self.n, tileNb)
        self.row_offsets = self._prefix(self.mt, tileMb)
        self.col_offsets = self._prefix(self.nt, tileNb)
        self.table = _host.TileTable()
        self.tiles = {}            # (i, j, slot) -> 2-D tensor (col-major view)
        self.local = {}            # slot -> contiguous local buffer (block-cyclic case)
        self.origin_slot = None
        self.lock = threading.RLock()
        self.pools = {}
        self.pool_chunks = {}
        self.pool_blocks = {}      # (i, j, slot) -> (chunk, idx)
        self.bc = self._detect_block_cyclic()

    # ------------------------------------------------------------------
    @staticmethod
    def _count_tiles(n, size):
        if n <= 0:
            return 0
        if getattr(size, "kind", None) == "uniform":
            return -(-n // size.nb)
        t, s = 0, 0
        while s < n:
            s += size(t)
            t += 1
        return t

    @staticmethod
    def _prefix(nt, size):
        off = [0]
        for i in range(nt):
            off.append(off[-1] + size(i))
        return off

    def _detect_block_cyclic(self) -> Optional[BlockCyclic]:
        if getattr(self.tileMb, "kind", None) != "uniform" or getattr(self.tileNb, "kind", None) != "uniform":
            return None
        tr = self.tileRank
        if getattr(tr, "kind", None) == "2d" and getattr(tr, "mb", 0) == 1 and getattr(tr, "nb", 0) == 1 and \
                tr.p * tr.q <= self.comm.size:
            # the grid the constructor asked for (also for matrices with a
            # single tile, whose ownership alone cannot reveal p x q)
            ok, order, p, q = True, tr.order, tr.p, tr.q
        else:
            ok, order, p, q = func.is_2d_cyclic_grid(self.mt, self.nt, self.tileRank)
        if not ok:
            return None
        if self.mt <= 1 and self.nt <= 1 and self.comm.size > 1 and getattr(tr, "kind", None) != "2d":
            # a single tile: rank from the function
            r = self.tileRank((0, 0)) if self.mt and self.nt else 0
            p = q = 1
            if r != 0:
                return None
        if p * q > self.comm.size:
            return None
        mb, nb = self.tileMb.nb, self.tileNb.nb
        me = self.rank
        if me < p * q and me >= 0:
            pr, pc = (me % p, me // p) if order == GridOrder.Col else (me // q, me % q)
            mloc, nloc = numroc(self.m, mb, pr, p), numroc(self.n, nb, pc, q)
        else:
            pr = pc = -1
            mloc = nloc = 0
        lld = max(1, -(-mloc // 16) * 16)
        return BlockCyclic(mb, nb, p, q, order, pr, pc, mloc, nloc, lld)

    # ------------------------------------------------------------------
    def slot_of(self, device) -> int:
        return DEV if torch.device(device).type == "cuda" else HOST

    def device_of(self, slot) -> torch.device:
        return self.device if slot == DEV else torch.device("cpu")

    def tileIsLocal(self, i, j) -> bool:
        return self.tileRank((i, j)) == self.rank

    def tile_shape(self, i, j):
        return self.tileMb(i), self.tileNb(j)

    # ---- allocation --------------------------------------------------
    def allocate_local(self, slot: int, buffer: Optional[torch.Tensor] = None, kind=TileKind.SlateOwned):
        """Create (or wrap) the contiguous local buffer and register local tiles."""
        bc = self.bc
        slate_assert(bc is not None, "allocate_local requires a block-cyclic storage")
        with self.lock:
            if buffer is None:
                dev = self.device_of(slot)
                buf = torch.zeros((bc.nloc, bc.lld), dtype=self.dtype, device=dev).t()
            else:
                buf = buffer
                slate_assert(buf.shape[0] >= bc.mloc and buf.shape[1] >= bc.nloc, "local buffer too small")
                slate_assert(buf.stride(0) == 1 or buf.shape[0] <= 1, "local buffer must be column-major")
                bc.lld = max(1, buf.stride(1))
            self.local[slot] = buf
            if self.origin_slot is None:
                self.origin_slot = slot
            origin = self.origin_slot == slot
            for j in (range(bc.pc, self.nt, bc.q) if bc.pc >= 0 else []):
                for i in range(bc.pr, self.mt, bc.p):
                    self.table.insert(i, j, slot, int(kind) if origin else 0, origin)
                    if not origin:
                        # mirror instance: valid only after a copy
                        self.table.set_state(i, j, slot, _host.MOSI_Invalid)
        return self.local[slot]

    def local_tile_view(self, slot, i, j) -> torch.Tensor:
        bc = self.bc
        buf = self.local[slot]
        li = (i // bc.p) * bc.mb
        lj = (j // bc.q) * bc.nb
        mb, nb = self.tileMb(i), self.tileNb(j)
        return buf[li:li + mb, lj:lj + nb]

    def _pool(self, slot):
        p = self.pools.get(slot)
        if p is None:
            mb = max((self.tileMb(i) for i in range(self.mt)), default=1)
            nb = max((self.tileNb(j) for j in range(self.nt)), default=1)
            elems = max(1, mb * nb)
            per_chunk = max(1, min(256, (1 << 28) // (elems * self._itemsize())))
            dev = self.device_of(slot)
            if dev.type == "cuda":
                import os
                cap = int(float(os.environ.get("SLATE_AMD_POOL_GIB", "0")) * (1 << 30))
                p = _native.hip().DevicePool(dev.index if dev.index is not None else torch.cuda.current_device(),
                                             elems * self._itemsize(), per_chunk, cap)
            else:
                p = _host.SlabPool(elems * self._itemsize(), per_chunk)
            self.pools[slot] = p
            self.pool_chunks[slot] = []
            self._pool_geom = (mb, nb)
        return p

    def pool_stats(self, slot=DEV) -> dict:
        """Occupancy of a slot's workspace pool (empty dict if none yet)."""
        p = self.pools.get(slot)
        if p is None:
            return {}
        if hasattr(p, "stats"):
            return dict(p.stats())
        return {"in_use": p.in_use(), "peak": p.peak(), "chunks": p.chunks(),
                "capacity": p.capacity(), "block_bytes": p.block_bytes()}

    def _itemsize(self):
        return torch.empty((), dtype=self.dtype).element_size()

    def _alloc_tile(self, i, j, slot, kind) -> torch.Tensor:
        mb, nb = self.tileMb(i), self.tileNb(j)
        if kind == TileKind.Workspace:
            pool = self._pool(slot)
            chunks = self.pool_chunks[slot]
            pmb, pnb = self._pool_geom
            dev = self.device_of(slot)
            if dev.type == "cuda":
                # stream-ordered native pool: blocks of block_bytes (>= tile bytes,
                # 256-byte aligned) inside hipMalloc'd chunks exported by DLPack
                chunk, idx, off, grew = pool.alloc(torch.cuda.current_stream(dev).cuda_stream)
                while len(chunks) <= chunk:
                    raw = torch.utils.dlpack.from_dlpack(pool.chunk_view(len(chunks)))
                    chunks.append(raw.view(self.dtype))
                per = pool.block_bytes() // self._itemsize()
                flat = chunks[chunk][idx * per: idx * per + mb * nb]
            else:
                chunk, idx, grew = pool.alloc()
                if grew:
                    chunks.append(torch.empty((pool.blocks_per_chunk(), pmb * pnb), dtype=self.dtype,
                                              device=dev))
                flat = chunks[chunk][idx, : mb * nb]
            self.pool_blocks[(i, j, slot)] = (chunk, idx)
            return flat.view(nb, mb).t() if mb > 0 and nb > 0 else flat.view(mb, nb)
        return torch.zeros((nb, max(mb, 1)), dtype=self.dtype, device=self.device_of(slot)).t()[:mb, :]

    def _free_tile(self, i, j, slot):
        blk = self.pool_blocks.pop((i, j, slot), None)
        if blk is not None:
            dev = self.device_of(slot)
            if dev.type == "cuda":
                # stream-ordered: reusable by this stream at once, by others
                # after its event.  A workspace tile may have been last read on
                # a pipeline stream (panel / diag / update) other than the
                # freeing one: the freeing stream first waits for all of them,
                # so the block cannot be handed out while one still reads it
                # (ADVICE r2).  Frees are rare (workspace release), the joins
                # cheap (event record + wait per stream).
                cur = torch.cuda.current_stream(dev)
                from ..parallel.streams import StreamSet
                for other in StreamSet.streams_of(dev):
                    if other is not None and other != cur:
                        cur.wait_event(other.record_event())
                self.pools[slot].free(*blk, cur.cuda_stream)
            else:
                self.pools[slot].free(*blk)
        self.tiles.pop((i, j, slot), None)

    def tileInsert(self, i, j, slot, data: Optional[torch.Tensor] = None, kind=TileKind.SlateOwned,
                   origin=None):
        """Insert a tile instance (allocated, user-provided, or workspace)."""
        with self.lock:
            if data is None:
                data = self._alloc_tile(i, j, slot, kind)
            self.tiles[(i, j, slot)] = data
            if origin is None:
                origin = kind != TileKind.Workspace
            self.table.insert(i, j, slot, int(kind), bool(origin))
            if origin and self.origin_slot is None:
                self.origin_slot = slot
            return data

    def tile_data(self, i, j, slot) -> Optional[torch.Tensor]:
        t = self.tiles.get((i, j, slot))
        if t is not None:
            return t
        if self.bc is not None and slot in self.local and self.tileIsLocal(i, j):
            return self.local_tile_view(slot, i, j)
        return None

    def tileExists(self, i, j, slot=None) -> bool:
        return self.table.exists(i, j, -1 if slot is None else slot)

    def tileErase(self, i, j, slot=None):
        with self.lock:
            slots = [HOST, DEV] if slot is None else [slot]
            for s in slots:
                if (i, j, s) in self.tiles:
                    self._free_tile(i, j, s)
                self.table.erase(i, j, s)

    def tileRelease(self, i, j, slot):
        with self.lock:
            if self.table.release(i, j, slot):
                self._free_tile(i, j, slot)

    # ---- coherency ---------------------------------------------------------
    def tileGet(self, i, j, slot, modify=False, hold=False) -> torch.Tensor:
        """Acquire tile (i,j) in memory space `slot` (BaseMatrix::tileGet)."""
        with self.lock:
            if not self.table.exists(i, j, slot) and self.tile_data(i, j, slot) is None:
                self.tileInsert(i, j, slot, kind=TileKind.Workspace, origin=False)
            elif not self.table.exists(i, j, slot):
                self.table.insert(i, j, slot, 0, False)
                self.table.set_state(i, j, slot, _host.MOSI_Invalid)
            src = self.table.acquire(i, j, slot, modify, hold)
            dst = self.tile_data(i, j, slot)
            if src >= 0:
                dst.copy_(self.tile_data(i, j, src), non_blocking=(slot == DEV))
            return dst

    def tileModified(self, i, j, slot, permissive=False):
        self.table.modified(i, j, slot, permissive)

    def tileState(self, i, j, slot) -> int:
        return self.table.state(i, j, slot)

    def tileUpdateOrigin(self, i, j):
        with self.lock:
            src = self.table.update_origin_source(i, j)
            if src >= 0:
                o = self.table.origin(i, j)
                self.tile_data(i, j, o).copy_(self.tile_data(i, j, src))

    def mark_local_modified(self, slot):
        """After a whole-local-buffer kernel wrote `slot` (the post-condition
        of every driver: with SLATE_AMD_DEBUG=1 the MOSI checker runs here)."""
        self.table.mark_all(slot, _host.MOSI_Modified)
        from ..utils.debug import Debug
        if Debug.enabled():
            Debug.assert_mosi(self, "mark_local_modified")

    def prepare_local(self, slot) -> torch.Tensor:
        """Make the contiguous local buffer valid in `slot` and return it."""
        bc = self.bc
        slate_assert(bc is not None, "prepare_local requires block-cyclic storage")
        with self.lock:
            if self.origin_slot is None:
                self.allocate_local(slot)
            if slot not in self.local:
                self.allocate_local(slot)
            other = HOST if slot == DEV else DEV
            need = False
            for (i, j, s) in self.table.instances():
                if s == slot and self.tileIsLocal(i, j) and \
                        (self.table.state(i, j, s) & 0x111) == _host.MOSI_Invalid:
                    need = True
                    break
            if need and other in self.local:
                # bulk copy of the whole local buffer, then fix individual
                # tiles whose latest copy is a separate workspace instance
                self.local[slot].copy_(self.local[other])
            for (i, j, s) in self.table.instances():
                if s == slot and self.tileIsLocal(i, j) and \
                        (self.table.state(i, j, s) & 0x111) == _host.MOSI_Invalid:
                    srcs = [x for x in (HOST, DEV) if x != slot and self.table.exists(i, j, x)
                            and (self.table.state(i, j, x) & 0x111) != _host.MOSI_Invalid]
                    if srcs:
                        sd = self.tile_data(i, j, srcs[0])
                        if sd is not None and not (other in self.local and need and
                                                   (i, j, srcs[0]) not in self.tiles):
                            self.local_tile_view(slot, i, j).copy_(sd)
                    self.table.set_state(i, j, slot, _host.MOSI_Shared)
            from ..utils.debug import Debug
            if Debug.enabled():
                Debug.assert_mosi(self, "prepare_local")
            return self.local[slot]

    def sync_origin(self):
        """tileUpdateAllOrigin for the whole storage."""
        with self.lock:
            if self.bc is not None and self.origin_slot is not None and len(self.local) > 1:
                o = self.origin_slot
                other = HOST if o == DEV else DEV
                stale = any(s == o and self.tileIsLocal(i, j) and
                            (self.table.state(i, j, s) & 0x111) == _host.MOSI_Invalid
                            for (i, j, s) in self.table.instances())
                if stale:
                    self.local[o].copy_(self.local[other])
                    self.table.mark_all(o, _host.MOSI_Shared)
                return
            for (i, j, s) in self.table.instances():
                if self.table.origin(i, j) == s:
                    self.tileUpdateOrigin(i, j)

    def clearWorkspace(self):
        with self.lock:
            for (i, j, s) in list(self.tiles.keys()):
                if not self.tileIsLocal(i, j):
                    self._free_tile(i, j, s)
            self.table.clear_workspace()

    def releaseWorkspace(self):
        self.clearWorkspace()
