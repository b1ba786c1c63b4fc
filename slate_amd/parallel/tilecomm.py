"""Tile-set transfers between ranks (SLATE `tileBcast`, `listBcast`,
`listBcastMT`, `listReduce`, `tileSend/Recv`: `include/slate/BaseMatrix.hh:
1762-2452`, hypercube patterns in `src/internal/internal_comm.cc:72-115`).

On a fully connected xGMI node the MI355X design does not build per-tile
radix-k trees.  Instead every transfer step is planned *deterministically on
all ranks* (who owns each tile, who needs it) and executed as ONE batched
point-to-point exchange (RCCL group of send/recv: every pair of GPUs uses
its own link concurrently), with the tiles of one (src, dst) pair packed
into a single contiguous message.
"""
from __future__ import annotations

import torch

from .. import ops


def exchange_tiles(comm, needs, owner_of, get_tile, shape_of, dtype, device):
    """Deliver tiles to the ranks that need them.

    needs:    dict rank -> list of tile keys that rank needs (same on all ranks)
    owner_of: key -> owning rank
    get_tile: key -> local 2-D column-major tensor (called on the owner)
    shape_of: key -> (rows, cols)
    Returns {key: tensor} for the keys this rank needs (own tiles are returned
    as views without copies)."""
    me = comm.rank
    out = {}
    sends, recvs, recv_layout = {}, {}, {}
    # what I send to each destination
    for dst, keys in needs.items():
        if dst == me:
            continue
        mine = [k for k in keys if owner_of(k) == me]
        if mine:
            tot = sum(shape_of(k)[0] * shape_of(k)[1] for k in mine)
            buf = torch.empty(tot, dtype=dtype, device=device)
            off = 0
            for k in mine:
                r, c = shape_of(k)
                t = get_tile(k)
                buf[off:off + r * c].view(c, r).t().copy_(t)
                off += r * c
            sends[dst] = buf
    # what I receive
    for k in needs.get(me, []):
        o = owner_of(k)
        if o == me:
            out[k] = get_tile(k)
        else:
            recv_layout.setdefault(o, []).append(k)
    for src, keys in recv_layout.items():
        tot = sum(shape_of(k)[0] * shape_of(k)[1] for k in keys)
        recvs[src] = torch.empty(tot, dtype=dtype, device=device)
    comm.exchange(sends, recvs)
    for src, keys in recv_layout.items():
        buf = recvs[src]
        off = 0
        for k in keys:
            r, c = shape_of(k)
            out[k] = buf[off:off + r * c].view(c, r).t()
            off += r * c
    return out


def bcast_tile(comm, tile: torch.Tensor, root: int):
    """Broadcast one (possibly strided) tile from comm-rank root."""
    if comm.size == 1:
        return tile
    if tile.is_contiguous() or (tile.stride(0) == 1 and tile.stride(1) == tile.shape[0]):
        comm.bcast(tile, root)
        return tile
    tmp = ops.colmajor_empty(tile.shape[0], tile.shape[1], tile.dtype, tile.device)
    if comm.rank == root:
        tmp.copy_(tile)
    comm.bcast(tmp, root)
    if comm.rank != root:
        tile.copy_(tmp)
    return tile
