"""Exact point-to-point row / column interchanges on block-cyclic local
buffers (SLATE internal::permuteRows / permuteRowsCols,
src/internal/internal_swap.cc): given the global moves (dst, src) -- the
new line dst holds the old line src -- only the lines that change owner
travel, one batched send/recv per peer, in dst order on both sides; the
lines that stay on their rank move locally."""
from __future__ import annotations

import numpy as np
import torch

from .. import ops


def moves_from_ipiv(ipiv, k0):
    """Moves of the LAPACK-style sequential interchanges ipiv (global,
    0-based) applied at rows k0, k0 + 1, ..."""
    cur = {}
    for i, t in enumerate(np.asarray(ipiv).tolist()):
        a, b = k0 + i, int(t)
        if a != b:
            ca, cb = cur.get(a, a), cur.get(b, b)
            cur[a], cur[b] = cb, ca
    return sorted((d, s) for d, s in cur.items() if d != s)


def moves_from_perm(perm):
    """Moves of new[i] = old[perm[i]]."""
    perm = np.asarray(perm)
    idx = np.nonzero(perm != np.arange(perm.size))[0]
    return [(int(i), int(perm[i])) for i in idx]


def exchange_lines(comm, data, moves, nb, p, me, axis=0):
    """Apply ``moves`` to the local lines of ``data``: axis 0 = rows (local
    row i of process index ``me`` over ``p`` processes, tile nb), axis 1 =
    columns.  ``comm`` ranks are the process indices along that axis.
    Returns the bytes this rank sent."""
    if not moves:
        return 0
    nl = data.shape[axis]
    w = data.shape[1 - axis]

    def own(g):
        return (g // nb) % p

    def loc(g):
        return (g // (nb * p)) * nb + g % nb

    sends, recvs, ld_, ls_ = {}, {}, [], []
    for d, s in moves:
        od, os_ = own(d), own(s)
        if os_ == me and od != me:
            sends.setdefault(od, []).append(loc(s))
        elif od == me and os_ != me:
            recvs.setdefault(os_, []).append(loc(d))
        elif od == me and os_ == me:
            ld_.append(loc(d))
            ls_.append(loc(s))
    if (not sends and not recvs and not ld_) or w == 0:
        return 0
    dev, dt = data.device, data.dtype
    peers_s, peers_r = sorted(sends), sorted(recvs)
    parts = [sends[r] for r in peers_s] + [recvs[r] for r in peers_r] + [ls_, ld_]
    flat = np.concatenate([np.asarray(x, dtype=np.int64) for x in parts])
    if flat.size and int(flat.max()) >= nl:
        raise IndexError(f"exchange_lines: local line {int(flat.max())} >= {nl}")
    idx = torch.from_numpy(flat)
    if data.is_cuda:
        idx = idx.pin_memory().to(dev, non_blocking=True)

    # device columns of 8 / 16-byte elements move by the column-copy kernel
    # (buffer = the c columns back to back); other cases by torch index ops
    kcols = data.is_cuda and data.element_size() in (8, 16) and data.stride(0) == 1

    def gather(ix):
        if axis == 0:
            t = torch.empty(w, ix.numel(), dtype=dt, device=dev)      # (w, c): column-major c x w
            ops.row_gather(data, t.t(), ix)
            return t
        if kcols:
            t = torch.empty(w, ix.numel(), dtype=dt, device=dev)
            ops.cols_move(data, t.view(ix.numel(), w).t(), ix)        # column j at offset j w
            return t
        return data.index_select(1, ix).contiguous()                  # (w, c): the c columns

    def scatter(buf, ix):
        if axis == 0:
            ops.row_scatter(buf.t(), data, ix)
        elif kcols:
            ops.cols_move(buf.view(ix.numel(), w).t(), data, ix, scatter=True)
        else:
            data.index_copy_(1, ix, buf)

    off, sb, rb, rofs, nbytes = 0, {}, {}, {}, 0
    es = torch.empty(0, dtype=dt).element_size()
    for r in peers_s:
        c = len(sends[r])
        sb[r] = gather(idx[off:off + c])
        nbytes += c * w * es
        off += c
    for r in peers_r:
        c = len(recvs[r])
        rb[r] = torch.empty(w, c, dtype=dt, device=dev)                # both axes: (line length, lines)
        rofs[r] = (off, c)
        off += c
    nloc = len(ls_)
    tmp = gather(idx[off:off + nloc]) if nloc else None
    if sb or rb:
        comm.exchange(sb, rb)
    for r in peers_r:
        o, c = rofs[r]
        scatter(rb[r], idx[o:o + c])
    if nloc:
        scatter(tmp, idx[off + nloc:off + 2 * nloc])
    return nbytes
