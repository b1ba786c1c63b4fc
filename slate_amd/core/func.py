"""Tile-size and tile-distribution functions (`include/slate/func.hh:39-334`).

A distribution is any callable ``f((i, j)) -> rank``; a tile-size function
is ``f(i) -> size``.  The closures returned here carry their parameters as
attributes (``.kind``, ``.p``, ``.q``, ``.order``, ``.nb``) so the storage
layer can recognise a 2D block-cyclic layout in O(1) and switch to the
contiguous ScaLAPACK-style local buffer (one GEMM launch per trailing
update) instead of a per-tile map.

On one MI355X node "rank" == GPU (one process per GPU), so the SLATE
distinction between process and device grids collapses: ``device_*``
variants are kept for API parity and compute the same functions.
"""
from __future__ import annotations

from .enums import GridOrder


def uniform_blocksize(n: int, nb: int):
    """Tiles of size nb, last one possibly smaller (func.hh:39-42)."""
    nt = max(1, -(-n // nb)) if n > 0 else 0
    last = n - (nt - 1) * nb if nt > 0 else 0

    def f(i):
        return nb if i < nt - 1 else last
    f.kind, f.nb, f.n = "uniform", nb, n
    return f


def max_blocksize(nt: int, size) -> int:
    return max((size(i) for i in range(nt)), default=0)


def _grid2d(order, mb, nb, p, q):
    order = GridOrder.from_string(order)
    if order == GridOrder.Unknown:
        raise ValueError("GridOrder.Unknown")
    if order == GridOrder.Col:
        def f(ij):
            i, j = ij
            return (i // mb) % p + ((j // nb) % q) * p
    else:
        def f(ij):
            i, j = ij
            return ((i // mb) % p) * q + (j // nb) % q
    f.kind = "2d" if (mb == 1 and nb == 1) else "2d_block"
    f.order, f.p, f.q, f.mb, f.nb = order, p, q, mb, nb
    return f


def device_2d_grid(order, m: int, n: int, p: int, q: int):
    """Blocks of m x n tiles dealt 2D-cyclically over a p x q grid."""
    return _grid2d(order, m, n, p, q)


def device_1d_grid(order, block_size: int, size: int):
    order = GridOrder.from_string(order)
    if order == GridOrder.Col:
        return _grid2d(order, block_size, 1, size, 1)
    return _grid2d(order, 1, block_size, 1, size)


def process_2d_grid(order, p: int, q: int):
    """Tile (i, j) -> rank on a p x q grid (func.hh:178-186)."""
    return _grid2d(order, 1, 1, p, q)


def process_1d_grid(order, size: int):
    order = GridOrder.from_string(order)
    if order == GridOrder.Col:
        return process_2d_grid(order, size, 1)
    return process_2d_grid(order, 1, size)


def transpose_grid(old):
    def f(ij):
        return old((ij[1], ij[0]))
    if getattr(old, "kind", None) == "2d":
        f.kind = "2d"
        f.order = GridOrder.Row if old.order == GridOrder.Col else GridOrder.Col
        f.p, f.q, f.mb, f.nb = old.q, old.p, 1, 1
    return f


def is_2d_cyclic_grid(mt: int, nt: int, func):
    """Detect a 2D cyclic distribution. Returns (ok, order, p, q)."""
    if mt == 0 or nt == 0 or (mt == 1 and nt == 1):
        return True, GridOrder.Col, 1, 1
    if getattr(func, "kind", None) == "2d":
        return True, func.order, func.p, func.q
    if mt == 1 or nt == 1:
        order = GridOrder.Col
    elif func((1, 0)) == 1:
        order = GridOrder.Col
    elif func((0, 1)) == 1:
        order = GridOrder.Row
    elif func((1, 0)) == 0 and func((0, 1)) == 0:
        order = GridOrder.Col
    else:
        return False, GridOrder.Unknown, -1, -1
    p = q = 0
    if order == GridOrder.Col:
        while p < mt and func((p, 0)) == p:
            p += 1
        while q < nt and func((0, q)) == q * p:
            q += 1
    else:
        while q < nt and func((0, q)) == q:
            q += 1
        while p < mt and func((p, 0)) == p * q:
            p += 1
    if p == 0 or q == 0:
        return False, GridOrder.Unknown, -1, -1
    ref = process_2d_grid(order, p, q)
    for i in range(mt):
        for j in range(nt):
            if func((i, j)) != ref((i, j)):
                return False, GridOrder.Unknown, -1, -1
    return True, order, p, q


def grid_shape(nprocs: int):
    """Default p x q: as square as possible with p <= q (test/test.cc:738-763)."""
    p = int(nprocs ** 0.5)
    while p > 1 and nprocs % p:
        p -= 1
    return p, nprocs // p
