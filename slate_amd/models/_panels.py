"""Panel movement primitives shared by the distributed drivers.

For a block-cyclic p x q grid, a tile column panel P (rows distributed over
the process rows like the matrix rows) is needed by a rank in two shapes:

* ``Prow`` -- the panel rows of *this process row* (every local row of the
  trailing matrix): one broadcast over the row communicator from the
  process column that owns the panel (SLATE's listBcast of A(i,k) to the
  row A(i, k+1:i), `src/potrf.cc:122-132`);
* ``Lcol`` -- the panel rows whose global index equals one of *this rank's
  local columns* (the transposed operand of herk/potrf/her2k updates):
  each process row contributes the rows it owns, one column-communicator
  broadcast per process row of exactly those rows, assembled in local
  column order by one row-gather kernel (SLATE's listBcast of A(i,k) down
  the column A(i:nt-1, i)).

Plans are computed once per driver call on the host and uploaded as one
index tensor, so no host->device copy happens inside the step loop.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import ops
from ._util import tiles_local_before


def _ranges(starts, lens):
    """Concatenation of arange(s, s + l) over (s, l) pairs (numpy, no loop)."""
    starts = np.asarray(starts, dtype=np.int64)
    lens = np.asarray(lens, dtype=np.int64)
    tot = int(lens.sum()) if lens.size else 0
    if tot == 0:
        return np.zeros(0, dtype=np.int64)
    first = np.cumsum(lens) - lens                  # output position of each range
    return np.repeat(starts - first, lens) + np.arange(tot, dtype=np.int64)


def _rows_plan(mbs, tfirst, tend, nb, p, q, pc, cols_from):
    """``mbs[j]`` = row count of tile j.  Returns (rows_of[r] arrays, total,
    order array): the local rows (relative to the local start of tile
    ``tfirst``) process row r contributes, and where each needed tile's rows
    land in the gathered buffer, in tile order."""
    need = np.arange(cols_from, tend, dtype=np.int64)
    need = need[need % q == pc]
    mb = np.asarray([mbs[j] for j in need.tolist()], dtype=np.int64)
    r_of = need % p
    rows_of, base, pos = {}, {}, 0
    start_in_r = np.zeros(need.size, dtype=np.int64)
    for r in range(p):
        sel = r_of == r
        base_r = tiles_local_before(tfirst, p, r) * nb
        lj = (need[sel] // p) * nb - base_r
        rows_of[r] = _ranges(lj, mb[sel])
        start_in_r[sel] = np.cumsum(mb[sel]) - mb[sel]
        base[r] = pos
        pos += int(rows_of[r].size)
    bases = np.asarray([base[r] for r in range(p)], dtype=np.int64)
    order = _ranges(bases[r_of] + start_in_r, mb) if need.size else np.zeros(0, dtype=np.int64)
    return rows_of, pos, order


def _append_plan(flat, rows_of, tot, order, p):
    """Append one plan's index arrays to ``flat`` (a list of arrays; its
    running length is flat[0])."""
    meta = {}
    for r in range(p):
        meta[r] = (flat[0], int(rows_of[r].size))
        flat.append(rows_of[r])
        flat[0] += int(rows_of[r].size)
    meta["order"] = (flat[0], int(order.size))
    flat.append(order)
    flat[0] += int(order.size)
    meta["tot"] = tot
    return meta


def _upload(flat, dev):
    arrs = flat[1:]
    cat = np.concatenate(arrs) if arrs else np.zeros(0, dtype=np.int64)
    if cat.size == 0:
        cat = np.zeros(1, dtype=np.int64)
    t = torch.from_numpy(cat)
    if torch.device(dev).type == "cuda":
        t = t.pin_memory().to(dev, non_blocking=True)
    return t


def plan_col_gather(tileMb, tfirst, tend, nb, p, q, pc, dev, cols_from=None):
    """Plan for assembling the rows of panel tiles j in [cols_from, tend)
    with j % q == pc from Prow buffers whose row 0 is the local start of tile
    ``tfirst`` on each process row.  Returns (meta, idx_tensor)."""
    cols_from = tfirst if cols_from is None else cols_from
    key = ("one", tfirst, tend, nb, p, q, pc, cols_from, _mb_sig(tileMb, tfirst, tend), str(dev))
    hit = _PLAN_CACHE.get(key)
    if hit is not None:
        return hit
    mbs = {j: tileMb(j) for j in range(tfirst, tend)}
    flat = [0]
    meta = _append_plan(flat, *_rows_plan(mbs, tfirst, tend, nb, p, q, pc, cols_from), p)
    out = (meta, _upload(flat, dev))
    _cache_put(key, out)
    return out


# Plans depend only on the geometry: cached across driver calls (the bench
# and every solver factor the same shape repeatedly).  Cached index tensors
# are read-only.
_PLAN_CACHE = {}
_PLAN_CACHE_MAX = 64


def _cache_put(key, val):
    if len(_PLAN_CACHE) >= _PLAN_CACHE_MAX:
        _PLAN_CACHE.pop(next(iter(_PLAN_CACHE)))
    _PLAN_CACHE[key] = val


def _mb_sig(tileMb, t0, t1):
    """Row-count signature of tiles [t0, t1): uniform runs compress to
    (first, last, count) so the key stays small."""
    if t1 <= t0:
        return ()
    first, last = tileMb(t0), tileMb(t1 - 1)
    if t1 - t0 <= 2 or all(tileMb(j) == first for j in range(t0 + 1, t1 - 1)):
        return (first, last, t1 - t0)
    return tuple(tileMb(j) for j in range(t0, t1))


def plan_col_gathers_steps(tileMb, g0, nt, nb, p, q, pc, dev, split=None):
    """One plan per factorization step t (potrf: the rows below the
    diagonal tile g0+t), all uploaded as ONE index tensor.  With ``split``
    = la, each step gets two plans: the lookahead tiles g+1 .. g+la (the
    critical path) and the rest (the trailing update, off the critical
    path).  Built with numpy range arithmetic and cached per geometry, so a
    repeated call costs a dictionary lookup (the round-2 list-of-ints build
    took ~40 ms per call at n = 32768 on a 2 x 4 grid)."""
    key = ("steps", g0, nt, nb, p, q, pc, split, _mb_sig(tileMb, g0, g0 + nt), str(dev))
    hit = _PLAN_CACHE.get(key)
    if hit is not None:
        return hit
    mbs = {j: tileMb(j) for j in range(g0, g0 + nt)}
    flat, metas = [0], []
    for t in range(nt):
        g = g0 + t
        if split is None:
            metas.append(_append_plan(flat, *_rows_plan(mbs, g + 1, g0 + nt, nb, p, q, pc, g + 1), p))
        else:
            e = min(g + 1 + split, g0 + nt)
            metas.append((_append_plan(flat, *_rows_plan(mbs, g + 1, e, nb, p, q, pc, g + 1), p),
                          _append_plan(flat, *_rows_plan(mbs, g + 1, g0 + nt, nb, p, q, pc, e), p)))
    idx = _upload(flat, dev)
    if split is None:
        out = [(m, idx) for m in metas]
    else:
        out = [((a, idx), (b, idx)) for a, b in metas]
    _cache_put(key, out)
    return out


def assemble_cols(plan, Prow, grid, p, kb, dtype, dev, comm=None):
    """Lcol (rows = this rank's local columns of the panel range); the
    column broadcasts go over ``comm`` (default the grid's column
    communicator)."""
    comm = comm or grid.col_comm
    m, idx = plan
    tot = m["tot"]
    Rbuf = ops.colmajor_empty(tot, kb, dtype, dev)
    pos = 0
    for r in range(p):
        o, cnt = m[r]
        if cnt:
            chunk = Rbuf[pos:pos + cnt]
            if grid.pr == r:
                ops.row_gather(Prow, chunk, idx[o:o + cnt])
            if p > 1:
                if chunk.is_contiguous() or cnt == 0:
                    comm.bcast(chunk, r)
                else:
                    tmp = ops.colmajor_empty(cnt, kb, dtype, dev)
                    if grid.pr == r:
                        tmp.copy_(chunk)
                    comm.bcast(tmp, r)
                    chunk.copy_(tmp)
        pos += cnt
    o, cnt = m["order"]
    Lcol = ops.colmajor_empty(cnt, kb, dtype, dev)
    if cnt:
        ops.row_gather(Rbuf, Lcol, idx[o:o + cnt])
    return Lcol


def row_bcast(grid, src, owner_pc, nrows, kb, dtype, dev):
    """Broadcast a local-rows panel (nrows x kb) from process column owner_pc
    over the row communicator; ``src`` is the owner's local view."""
    if grid is None or grid.q == 1:
        return src
    P = ops.colmajor_empty(nrows, kb, dtype, dev)
    if grid.pc == owner_pc and nrows:
        P.copy_(src)
    if nrows:
        grid.row_comm.bcast(P, owner_pc)
    return P


def col_bcast(grid, src, owner_pr, kb, ncols, dtype, dev):
    """Broadcast a local-cols row panel (kb x ncols) from process row owner_pr
    over the column communicator."""
    if grid is None or grid.p == 1:
        return src
    P = ops.colmajor_empty(kb, ncols, dtype, dev)
    if grid.pr == owner_pr and ncols:
        P.copy_(src)
    if ncols:
        grid.col_comm.bcast(P, owner_pr)
    return P


_GROWS = {}


def rows_global(lr0, lr1, nb, p, pr, r0, dev):
    """Panel-relative global rows (global - r0) of local rows [lr0, lr1) of
    process row pr (block-cyclic, tile nb).  The local->global row table is
    uploaded once per (nb, p, pr, device) and sliced on the device, so the
    step loops of getrf / he2hb issue no host->device copy (the round-2
    version built and uploaded a fresh numpy range per step: a pageable copy
    that blocked the host until the stream caught up)."""
    key = (nb, p, pr, str(dev))
    tab = _GROWS.get(key)
    if tab is None or tab.numel() < lr1:
        L = max(lr1, 2 * (tab.numel() if tab is not None else 0), 1024)
        lr = np.arange(L, dtype=np.int64)
        g = torch.from_numpy(((lr // nb) * p + pr) * nb + lr % nb)
        if torch.device(dev).type == "cuda":
            g = g.pin_memory().to(dev, non_blocking=True)
        _GROWS[key] = tab = g
    if not r0:
        return tab[lr0:lr1]
    # shifted rows: formed on the host and uploaded pinned / non-blocking (a
    # device subtraction would be torch compute in the step loop)
    lr = np.arange(lr0, lr1, dtype=np.int64)
    g = torch.from_numpy(((lr // nb) * p + pr) * nb + lr % nb - r0)
    if torch.device(dev).type == "cuda":
        g = g.pin_memory().to(dev, non_blocking=True)
    return g


def panel_allgather(colc, buf, mloc, t0, lc, kb, nb, p, pr, nloc_r, dt, dev):
    """All-gather the rows at/after global tile t0 of the local columns
    [lc, lc + kb) inside the process column; returns (P, myidx): P holds the
    panel rows in GLOBAL order (row 0 = first row of tile t0), myidx the
    panel rows of this rank's local rows (for the write-back)."""
    cnt = [max(0, nloc_r[r] - min(tiles_local_before(t0, p, r) * nb, nloc_r[r])) for r in range(p)]
    lr0 = min(tiles_local_before(t0, p, pr) * nb, mloc)
    nmine = mloc - lr0
    r0 = t0 * nb
    mx = max(max(cnt), 1)
    pad = ops.colmajor_zeros(mx, kb, dt, dev)
    if nmine:
        pad[:nmine].copy_(buf[lr0:mloc, lc:lc + kb])
    allp = colc.allgather(pad.t()) if p > 1 else pad.t().unsqueeze(0)
    P = ops.colmajor_empty(sum(cnt), kb, dt, dev)
    for r in range(p):
        if cnt[r]:
            a = tiles_local_before(t0, p, r) * nb
            ops.row_scatter(allp[r].t()[:cnt[r]], P, rows_global(a, a + cnt[r], nb, p, r, r0, dev))
    myidx = rows_global(lr0, mloc, nb, p, pr, r0, dev)
    return P, myidx
