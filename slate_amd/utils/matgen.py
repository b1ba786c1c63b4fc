"""Matrix generator (`slate_matgen`: include/slate/generate_matrix.hh:17-75,
matgen/random.cc:36-60, matgen/generate_matrix_utils.cc).

Entries are a pure function of (seed, global i, global j) via a
counter-based Philox4x32-10 stream shared by the host runtime and the gfx950
kernel, so the same matrix is produced for any grid / tile size / device,
and a rank fills its local buffer on the GPU without host staging.
"""
from __future__ import annotations

from .. import ops
from ..core.exceptions import SlateError
from ..core.storage import DEV

KINDS = {
    "zeros": 0, "zero": 0, "ones": 1, "identity": 2, "ij": 3, "jordan": 4,
    "rand": 10, "rands": 11, "randn": 12, "randb": 13, "randr": 14,
    "rand_dominant": 20, "diag_dominant": 20, "poev": 21, "spd": 21, "hpd": 21,
    "heev": 22, "rands_hermitian": 22,
    "minij": 30, "hilb": 31, "lehmer": 32, "frank": 33, "moler": 34,
}


class MatgenParams:
    """SLATE MatgenParams subset: kind, seed, scale."""

    def __init__(self, kind="rands", seed=42, scale=1.0):
        self.kind, self.seed, self.scale = kind, seed, scale


def generate_matrix(A, kind="rands", seed=42, scale=1.0):
    """Fill every local tile of A (any view of a block-cyclic matrix).

    Kinds: zeros ones identity ij jordan rand rands randn randb randr
    rand_dominant (rands + max(m,n) I), poev/spd/hpd (Hermitian rands +
    n I, positive definite), heev (Hermitian rands), minij hilb lehmer frank
    moler (Matlab gallery)."""
    if isinstance(kind, MatgenParams):
        kind, seed, scale = kind.kind, kind.seed, kind.scale
    k = KINDS.get(str(kind).lower())
    if k is None:
        raise SlateError(f"unknown matrix kind {kind!r}")
    s = A.storage
    bc = s.bc
    if bc is None:
        # per-tile storage: generate tile by tile with its global offsets
        for (i, j, slot) in list(s.tiles.keys()):
            t = s.tiles[(i, j, slot)]
            ops.matgen(k, seed, t, s.m, s.n, max(t.shape[0], 1), 1, 0, max(t.shape[1], 1), 1, 0,
                       s.row_offsets[i], s.col_offsets[j], scale)
            s.table.modified(i, j, slot, True)
        return A
    if not s.local:
        A.insertLocalTiles(device=s.device if s.device.type == "cuda" else -1)
    slot = s.origin_slot
    buf = s.local[slot]
    if bc.pr < 0:
        return A
    R0, C0 = A.global_offsets()
    lb = A.local_block(slot)
    # generate the view's local block with its absolute global coordinates;
    # indices are offsets into the full matrix so the result matches any view
    ops.matgen(k, seed, lb.data, s.m, s.n, bc.mb, bc.p, bc.pr, bc.nb, bc.q, bc.pc, 0, 0, scale) \
        if (lb.row_off == 0 and lb.col_off == 0) else \
        _gen_offset(k, seed, lb, s, bc, scale)
    s.mark_local_modified(slot)
    return A


def _gen_offset(k, seed, lb, s, bc, scale):
    # local block starting at local (row_off, col_off): the kernel's
    # local->global map assumes local index 0 at tile start, so generate the
    # enclosing tile-aligned block and copy the needed part.
    r_al = (lb.row_off // bc.mb) * bc.mb
    c_al = (lb.col_off // bc.nb) * bc.nb
    full = s.local[s.origin_slot]
    big = full[r_al:lb.row_off + lb.mloc, c_al:lb.col_off + lb.nloc]
    tmp = ops.colmajor_empty(big.shape[0], big.shape[1], big.dtype, big.device)
    # global of local r_al: l2g(r_al) = ((r_al/mb)*p + pr)*mb -> pass as row0 with a 1-tile-per-proc map
    from ..core.storage import l2g
    ops.matgen(k, seed, tmp, s.m, s.n, bc.mb, bc.p, bc.pr, bc.nb, bc.q, bc.pc,
               l2g(r_al, bc.mb, bc.pr, bc.p) - bc.pr * bc.mb, l2g(c_al, bc.nb, bc.pc, bc.q) - bc.pc * bc.nb,
               scale)
    lb.data.copy_(tmp[lb.row_off - r_al:, lb.col_off - c_al:])
