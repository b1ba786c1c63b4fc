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

import torch

from .. import ops
from ._util import tiles_local_before


def _rows_plan(tileMb, tfirst, tend, nb, p, q, pc, cols_from):
    need = [j for j in range(cols_from, tend) if j % q == pc]
    rows_of = {}
    for r in range(p):
        base_r = tiles_local_before(tfirst, p, r) * nb
        idx = []
        for j in need:
            if j % p != r:
                continue
            lj = (j // p) * nb - base_r
            idx.extend(range(lj, lj + tileMb(j)))
        rows_of[r] = idx
    base, pos = {}, 0
    for r in range(p):
        base[r] = pos
        pos += len(rows_of[r])
    order = []
    cursor = {r: 0 for r in range(p)}
    for j in need:
        r = j % p
        rows = tileMb(j)
        order.extend(range(base[r] + cursor[r], base[r] + cursor[r] + rows))
        cursor[r] += rows
    return rows_of, pos, order


def _append_plan(flat, rows_of, tot, order, p):
    meta = {}
    for r in range(p):
        meta[r] = (len(flat), len(rows_of[r]))
        flat.extend(rows_of[r])
    meta["order"] = (len(flat), len(order))
    flat.extend(order)
    meta["tot"] = tot
    return meta


def plan_col_gather(tileMb, tfirst, tend, nb, p, q, pc, dev, cols_from=None):
    """Plan for assembling the rows of panel tiles j in [cols_from, tend)
    with j % q == pc from Prow buffers whose row 0 is the local start of tile
    ``tfirst`` on each process row.  Returns (meta, idx_tensor)."""
    cols_from = tfirst if cols_from is None else cols_from
    flat = []
    meta = _append_plan(flat, *_rows_plan(tileMb, tfirst, tend, nb, p, q, pc, cols_from), p)
    return meta, torch.tensor(flat if flat else [0], dtype=torch.int64, device=dev)


def plan_col_gathers_steps(tileMb, g0, nt, nb, p, q, pc, dev, split=None):
    """One plan per factorization step t (potrf: the rows below the
    diagonal tile g0+t), all uploaded as ONE index tensor.  With ``split``
    = la, each step gets two plans: the lookahead tiles g+1 .. g+la (the
    critical path) and the rest (the trailing update, off the critical
    path)."""
    flat, metas = [], []
    for t in range(nt):
        g = g0 + t
        if split is None:
            metas.append(_append_plan(flat, *_rows_plan(tileMb, g + 1, g0 + nt, nb, p, q, pc, g + 1), p))
        else:
            e = min(g + 1 + split, g0 + nt)
            metas.append((_append_plan(flat, *_rows_plan(tileMb, g + 1, e, nb, p, q, pc, g + 1), p),
                          _append_plan(flat, *_rows_plan(tileMb, g + 1, g0 + nt, nb, p, q, pc, e), p)))
    idx = torch.tensor(flat if flat else [0], dtype=torch.int64, device=dev)
    if split is None:
        return [(m, idx) for m in metas]
    return [((a, idx), (b, idx)) for a, b in metas]


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


def rows_global(lr0, lr1, nb, p, pr, r0, dev):
    """Panel-relative global rows (global - r0) of local rows [lr0, lr1) of
    process row pr (block-cyclic, tile nb)."""
    import numpy as np
    lr = np.arange(lr0, lr1, dtype=np.int64)
    g = ((lr // nb) * p + pr) * nb + lr % nb - r0
    return torch.from_numpy(g).to(dev)


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
