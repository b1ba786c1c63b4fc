"""Divide & conquer for the symmetric tridiagonal eigenproblem, with the
eigenvector matrix distributed by ROWS over the ranks.

Reference: src/stedc.cc, stedc_solve.cc:79-238 (recursion, OpenMP tasks),
stedc_merge.cc, stedc_deflate.cc:366-379, stedc_secular.cc:132,148,
stedc_z_vector.cc:94 (MPI_Allreduce of z-hat), stedc_sort.cc; LAPACK
laed1-laed4 (laed3's two half GEMMs).

MI355X design
* Q, the accumulated eigenvector matrix, is 1-D distributed: rank r owns
  the contiguous rows [r0, r1) of every column (a block of ~n/P rows).
  A merge of the subproblems [a, m) and [m, b) is Q[:, a:b] <- Q[:, a:b] V
  with V the rank-one eigenvector matrix, so every rank updates ITS rows
  with no communication of Q at all; the only data that travels per tree
  level is one all-reduce of 2n doubles: the children's eigenvalues and
  the boundary rows that form z (the reference's Allreduce of z /
  Allgatherv of lambda).  No rank holds an n x n matrix (the final
  row -> column redistribution for the back-transforms is one batched p2p
  exchange, parallel/redist.py).
* Leaves (<= 128 rows on the GPU, 64 on the host) are solved all at once on
  the GPU: one workgroup per leaf, implicit QL with each thread owning a
  row of the leaf's vectors (csrc/hip/stedc.hip steqr_leaf_kernel).
* Per merge: sort (device argsort), deflation by the tolerance test
  (device) and close-pole Givens chains (one thread per run,
  stedc_runs_kernel; rotations applied to the rows by rot_cols_kernel),
  secular roots / z-hat (wave-per-root kernels), the rank-one vectors in
  column chunks straight into the GEMM operand, and laed3's split GEMM:
  the rows of the top child only meet the columns that are nonzero there
  (top or rotation-mixed), the bottom rows likewise -- about half the flops
  of one dense product.
* The recursion is processed level by level (all merges of one depth
  before the next), the reference's task parallelism, expressed as a fixed
  bottom-up schedule.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .. import ops
from .._native import hip as _hip
from ..core.exceptions import SlateError
from ..utils.trace import trace_block

LEAF = 64
# leaves solved on the GPU (steqr_leaf_kernel, <= 128 rows): 128 halves the
# merges of the first level (SLATE_AMD_STEDC_LEAF = 64 keeps one wave each)
GPU_LEAF = min(128, max(16, int(os.environ.get("SLATE_AMD_STEDC_LEAF", "128"))))
CHUNK = 4096          # rank-one vector columns formed per merge GEMM


def _tree(n, leaf=LEAF):
    """(leaves, levels): leaves = [(a, b)], levels[t] = merges (a, m, b) at
    depth t (t = 0 is the root).  Split at the middle, as LAPACK."""
    leaves, levels = [], []

    def rec(a, b, t):
        if b - a <= leaf:
            leaves.append((a, b))
            return
        m = a + (b - a) // 2
        while len(levels) <= t:
            levels.append([])
        levels[t].append((a, m, b))
        rec(a, m, t + 1)
        rec(m, b, t + 1)

    if n > 0:
        rec(0, n, 0)
    return leaves, levels


def _split_diag(d, e, levels):
    """The leaves' diagonals: each split subtracts |rho| = e[m-1] from the
    two diagonal entries next to it (Cuppen's tear)."""
    d = d.copy()
    for lev in levels:
        for (a, m, b) in lev:
            rho = e[m - 1]
            d[m - 1] -= rho
            d[m] -= rho
    return d


def _row_range(n, P, r):
    mb = -(-n // P) if P else n
    return min(r * mb, n), min((r + 1) * mb, n), mb


def stedc_rows(d, e, comm=None, device=None, leaf=None):
    """Eigenvalues (ascending, host fp64, on every rank) and this rank's
    block of rows of the eigenvector matrix: returns (w, Qloc, r0, r1, mb)
    with Qloc (r1 - r0) x n column-major on ``device``; rank r owns rows
    [r * mb, (r + 1) * mb)."""
    dev = torch.device(device) if device is not None else torch.device("cpu")
    d = np.ascontiguousarray(np.asarray(d, dtype=np.float64).reshape(-1))
    e = np.ascontiguousarray(np.asarray(e, dtype=np.float64).reshape(-1))
    n = d.size
    P = comm.size if comm is not None else 1
    r = comm.rank if comm is not None else 0
    r0, r1, mb = _row_range(n, P, r)
    Q = ops.colmajor_zeros(r1 - r0, n, torch.float64, dev)
    w = torch.zeros(n, dtype=torch.float64, device=dev)
    if n == 0:
        return w.cpu(), Q, r0, r1, mb
    with trace_block("stedc"):
        # GPU leaves: up to GPU_LEAF rows (one workgroup each, stedc.hip);
        # host leaves: LEAF
        cap = GPU_LEAF if dev.type == "cuda" else LEAF
        leaves, levels = _tree(n, cap if leaf is None else min(int(leaf), cap))
        dl = _split_diag(d, e, levels)
        own = [(a, b) for (a, b) in leaves if a < r1 and b > r0] if P > 1 else leaves
        fails = _leaves(own, dl, e, w, Q, r0, r1, dev)
        ws = _LevelWork(n, dev) if dev.type == "cuda" else None
        for t in range(len(levels) - 1, -1, -1):
            mine = [(a, m, b) for (a, m, b) in levels[t] if a < r1 and b > r0]
            W, Z = _level_inputs(levels[t], w, Q, r0, r1, comm, dev)
            if ws is not None:
                _merge_level_gpu(mine, e, W, Z, w, Q, r0, r1, ws)
                continue
            for (a, m, b) in mine:
                _merge(a, m, b, float(e[m - 1]), W, Z, w, Q, r0, r1, dev)
        _check_leaves(fails, comm if P > 1 else None)
    return w.cpu(), Q, r0, r1, mb


def _leaves(own, dl, e, w, Q, r0, r1, dev):
    if not own:
        return
    if dev.type == "cuda":
        lo = torch.tensor([a for a, _ in own], dtype=torch.int64).pin_memory().to(dev, non_blocking=True)
        hi = torch.tensor([b for _, b in own], dtype=torch.int64).pin_memory().to(dev, non_blocking=True)
        dd = torch.from_numpy(dl).pin_memory().to(dev, non_blocking=True)
        ee = torch.from_numpy(np.concatenate([e, [0.0]])).pin_memory().to(dev, non_blocking=True)
        fails = torch.zeros(1, dtype=torch.int64, device=dev)
        import os
        _hip().steqr_leaves(len(own), lo.data_ptr(), hi.data_ptr(), dd.data_ptr(), ee.data_ptr(), w.data_ptr(),
                            Q.data_ptr(), max(1, Q.stride(1)), r0, r1, fails.data_ptr(),
                            torch.cuda.current_stream(dev).cuda_stream, max(b - a for a, b in own),
                            int(os.environ.get("SLATE_AMD_STEQR_MAXIT", "60")))
        return fails
    nfail = 0
    from .eig import steqr
    for (a, b) in own:
        try:
            wl, Zl = steqr(torch.from_numpy(dl[a:b].copy()), torch.from_numpy(e[a:b - 1].copy()))
        except SlateError:
            nfail += 1
            continue
        w[a:b] = wl
        lo, hi = max(a, r0), min(b, r1)
        if hi > lo:
            Q[lo - r0:hi - r0, a:b] = Zl[lo - a:hi - a, :].to(Q.dtype)
    return torch.tensor([nfail], dtype=torch.int64)


def _check_leaves(fails, comm):
    """a leaf whose QL iteration did not converge leaves wrong
    eigenpairs behind -- read the device counter once at the end (pinned,
    non-blocking: no extra sync point inside the D&C), reduce it over the
    ranks and fail like LAPACK stedc (info > 0) instead of returning them."""
    from ._util import read_to_host
    nf = int(read_to_host(fails)[0]) if fails is not None else 0
    if comm is not None and comm.size > 1:
        nf = int(comm.allreduce_scalar(nf, "max", torch.int64))
    if nf:
        from ..core.exceptions import NumericalError
        raise NumericalError(f"stedc: {nf} leaf eigenproblem(s) did not converge", nf)


def _level_inputs(merges, w, Q, r0, r1, comm, dev):
    """Children eigenvalues W[a:b] and z Z[a:b] (last row of the top child's
    vectors, first row of the bottom child's) of every merge at this depth,
    summed over ranks: each entry has exactly one writer (the owner of row
    a for W, of rows m-1 / m for Z)."""
    n = w.numel()
    buf = torch.zeros(2, n, dtype=torch.float64, device=dev)
    W, Z = buf[0], buf[1]
    P = comm.size if comm is not None else 1
    for (a, m, b) in merges:
        # each child's eigenvalues from the owner of its first row, the
        # boundary rows from their owners
        if P == 1 or r0 <= a < r1:
            W[a:m] = w[a:m]
        if P == 1 or r0 <= m < r1:
            W[m:b] = w[m:b]
        if r0 <= m - 1 < r1:
            Z[a:m] = Q[m - 1 - r0, a:m]
        if r0 <= m < r1:
            Z[m:b] = Q[m - r0, m:b]
    if P > 1:
        comm.allreduce(buf)
    return W, Z


# On a GPU every merge level runs the level-batched device merge
# (_merge_level_gpu: slate_hip kernels only).  The per-merge driver _merge
# below is the HOST path (CPU devices: gloo tests, host-only builds); it is
# never used for device-resident Q.
# host round trips of the last stedc_rows call (tests)
STEDC_STATS = {"host_syncs": 0, "levels": 0}


class _LevelWork:
    """Level-sized device arrays of the device merges (one slice [a, b) per
    merge), allocated once per stedc call."""

    def __init__(self, n, dev):
        f64 = dict(dtype=torch.float64, device=dev)
        i64 = dict(dtype=torch.int64, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        nn = max(n, 1)
        self.dd, self.zs, self.cs, self.sn, self.rC, self.rS, self.lam = (torch.empty(nn, **f64) for _ in range(7))
        self.ty, self.keep, self.rot = (torch.empty(nn, **i32) for _ in range(3))
        (self.order, self.c, self.K, self.S1, self.KS1, self.S2, self.KS2, self.D, self.isK, self.rI, self.rJ,
         self.o2) = (torch.empty(nn, **i64) for _ in range(12))
        self.dev = dev
        self.meta_bytes = int(_hip().stedc_meta_bytes())
        STEDC_STATS["host_syncs"] = 0
        STEDC_STATS["levels"] = 0

    def p(self, t, off=0):
        return t.data_ptr() + off * t.element_size()


def _merge_level_gpu(mine, e, W, Z, w, Q, r0, r1, ws):
    """All merges of one tree level with the sort, deflation, close-pole
    rotations and every index set formed on the device (stedc_level_prep,
    csrc/hip/stedc.hip); ONE host read of the per-merge sizes, then per
    merge: the rotations, the secular solve, laed3's split GEMM in CHUNK
    column blocks and the final ordering (a two-list merge of the roots and
    the deflated poles) -- all slate_hip kernels, no torch compute."""
    if not mine:
        return
    H = _hip()
    dev = ws.dev
    st = torch.cuda.current_stream(dev).cuda_stream
    nm = len(mine)
    rhos = [float(e[m - 1]) for (_, m, _) in mine]
    desc_h = np.asarray([(a, m, b, 1 if r < 0 else 0) for (a, m, b), r in zip(mine, rhos)], dtype=np.int64)
    desc = _upload(desc_h.reshape(-1), dev)
    rho_t = torch.from_numpy(np.abs(np.asarray(rhos, dtype=np.float64))).pin_memory().to(dev, non_blocking=True)
    meta = torch.empty(nm * ws.meta_bytes, dtype=torch.uint8, device=dev)
    maxs = max(b - a for (a, _, b) in mine)
    n = W.numel()
    H.stedc_level_prep(n, nm, maxs, desc.data_ptr(), rho_t.data_ptr(), W.data_ptr(), Z.data_ptr(), ws.p(ws.dd),
                       ws.p(ws.zs), ws.p(ws.ty), ws.p(ws.order), ws.p(ws.c), ws.p(ws.keep), ws.p(ws.rot),
                       ws.p(ws.cs), ws.p(ws.sn), meta.data_ptr(), ws.p(ws.K), ws.p(ws.S1), ws.p(ws.KS1),
                       ws.p(ws.S2), ws.p(ws.KS2), ws.p(ws.D), ws.p(ws.isK), ws.p(ws.rI), ws.p(ws.rJ),
                       ws.p(ws.rC), ws.p(ws.rS), st)
    from ._util import read_to_host
    mh = read_to_host(meta).numpy().view(np.uint8)          # the level's one host round trip
    STEDC_STATS["host_syncs"] += 1
    STEDC_STATS["levels"] += 1
    rec = mh.reshape(nm, ws.meta_bytes)
    ints = rec[:, :64].copy().view(np.int64).reshape(nm, 8)
    dbl = rec[:, 64:80].copy().view(np.float64).reshape(nm, 2)
    ldq = max(1, Q.stride(1))
    for t, ((a, m, b), rho) in enumerate(zip(mine, rhos)):
        _, k, nrot, n1, n2, nd = (int(x) for x in ints[t, :6])
        zzK = float(dbl[t, 1])
        flip = 1 if rho < 0 else 0
        r = abs(rho)
        s = b - a
        lo, hi = max(a, r0), min(b, r1)
        nr = hi - lo
        qm = Q.data_ptr() + ((lo - r0) + a * ldq) * 8            # Q[lo - r0, a]
        Qs = ops.colmajor_empty(nr, s, torch.float64, dev)
        H.cols_copy(nr, s, qm, ldq, ws.p(ws.order, a), Qs.data_ptr(), max(1, nr), 0, st)
        if nrot and nr:
            H.rot_cols(nr, Qs.data_ptr(), max(1, nr), nrot, ws.p(ws.rI, a), ws.p(ws.rJ, a), ws.p(ws.rC, a),
                       ws.p(ws.rS, a), st)
        dK = torch.empty(max(k, 1), dtype=torch.float64, device=dev)
        org = torch.empty(max(k, 1), dtype=torch.int64, device=dev)
        mu = torch.empty(max(k, 1), dtype=torch.float64, device=dev)
        if k:
            zK = torch.empty(k, dtype=torch.float64, device=dev)
            zh = torch.empty(k, dtype=torch.float64, device=dev)
            H.vec_gather(k, ws.p(ws.dd, a), ws.p(ws.K, a), dK.data_ptr(), st)
            H.vec_gather(k, ws.p(ws.zs, a), ws.p(ws.K, a), zK.data_ptr(), st)
            H.stedc_secular(k, dK.data_ptr(), zK.data_ptr(), r, zzK, org.data_ptr(), mu.data_ptr(), zh.data_ptr(),
                            0, 0, st)
        H.stedc_lambda(s, ws.p(ws.dd, a), ws.p(ws.isK, a), dK.data_ptr(), org.data_ptr(), mu.data_ptr(), flip,
                       ws.p(ws.lam, a), st)
        if k and nr:
            _merge_gemm_dev(H, ws, Qs, nr, a, k, lo, m, hi, n1, n2, dK, zh, org, mu, st)
        H.stedc_merge2(ws.p(ws.lam, a), ws.p(ws.K, a), k, ws.p(ws.D, a), nd, flip, ws.p(ws.o2, a), st)
        H.vec_gather(s, ws.p(ws.lam, a), ws.p(ws.o2, a), w.data_ptr() + a * 8, st)
        H.cols_copy(nr, s, Qs.data_ptr(), max(1, nr), ws.p(ws.o2, a), qm, ldq, 0, st)


def _merge_gemm_dev(H, ws, Qs, nr, a, k, lo, m, hi, n1, n2, dK, zh, org, mu, st):
    """Qs[:, K] <- Qs[:, K] V in CHUNK column blocks, the rows above m with
    the K columns nonzero there (S1 / KS1), the rows below with S2 / KS2
    (the device-built sets of stedc_compact_kernel)."""
    dev = ws.dev
    parts = []
    if lo < m:
        parts.append((0, min(hi, m) - lo, n1, ws.S1, ws.KS1))
    if hi > m:
        parts.append((max(lo, m) - lo, nr, n2, ws.S2, ws.KS2))
    srcs = []
    for (ra, rb, ns, S, KS) in parts:
        if ns == 0:
            srcs.append(None)
            continue
        Ap = ops.colmajor_empty(rb - ra, ns, torch.float64, dev)
        H.cols_copy(rb - ra, ns, Qs.data_ptr() + ra * 8, max(1, nr), ws.p(KS, a), Ap.data_ptr(), max(1, rb - ra), 0,
                    st)
        srcs.append(Ap)
    for j0 in range(0, k, CHUNK):
        nc = min(CHUNK, k - j0)
        V = ops.colmajor_empty(k, nc, torch.float64, dev)
        H.stedc_vectors(k, dK.data_ptr(), zh.data_ptr(), org.data_ptr(), mu.data_ptr(), j0, nc, V.data_ptr(),
                        max(1, k), st)
        for (ra, rb, ns, S, KS), Ap in zip(parts, srcs):
            out = ops.colmajor_empty(rb - ra, nc, torch.float64, dev)
            if Ap is not None:
                Vp = ops.colmajor_empty(ns, nc, torch.float64, dev)
                ops.row_gather(V, Vp, S[a:a + ns])
                ops.gemm(1.0, Ap, Vp, 0.0, out)
            else:
                ops.geset(0.0, 0.0, out)
            H.cols_copy(rb - ra, nc, out.data_ptr(), max(1, rb - ra), ws.p(ws.K, a + j0), Qs.data_ptr() + ra * 8,
                        max(1, nr), 1, st)


def _merge(a, m, b, rho, W, Z, w, Q, r0, r1, dev):
    """One merge on this rank's rows of [a, b) (HOST path: CPU tensors; the
    GPU runs _merge_level_gpu): see the module docstring."""
    if dev.type != "cpu":
        raise SlateError("stedc: the per-merge host path takes CPU tensors (GPU merges are level-batched)")
    s = b - a
    dd = W[a:b].clone()
    z = Z[a:b].clone()
    lo, hi = max(a, r0), min(b, r1)
    nr = hi - lo
    Qm = Q[lo - r0:hi - r0, a:b] if nr > 0 else None
    if rho == 0.0:
        o = torch.argsort(dd, stable=True)
        w[a:b] = dd[o]
        if nr:
            Q[lo - r0:hi - r0, a:b] = Qm[:, o].clone()
        return
    flip = rho < 0
    if flip:
        dd, rho = -dd, -rho
    # ---- sort poles ascending; types: 1 = top child column, 2 = bottom
    order = torch.argsort(dd, stable=True)
    dd = dd[order].contiguous()
    z = z[order].contiguous()
    ty = torch.where(order < (m - a), 1, 2).to(torch.int32)
    Qs = ops.colmajor_empty(nr, s, torch.float64, dev)
    if nr:
        Qs.copy_(Qm[:, order])
    # ---- deflation: tiny z components, then close-pole Givens chains.
    # Two host round trips per merge: (poles, z) for the tolerance test, then
    # (z after the rotations, rotation / keep flags, column types) -- every
    # index set is formed on the host and uploaded (pinned, stream-ordered)
    eps = float(np.finfo(np.float64).eps)
    hz = torch.cat([dd, z]).cpu().numpy()                                   # host sync 1
    dd_h, z_h = hz[:s], hz[s:]
    zz = float(np.dot(z_h, z_h))
    tolf = 8.0 * eps * max(float(np.abs(dd_h).max()), rho * zz)
    c_h = np.nonzero(~(rho * np.abs(z_h) * (zz ** 0.5) <= tolf))[0]
    nn = c_h.size
    c = _upload(c_h, dev)
    K_h = c_h
    ty_h = None
    z2_h = z_h
    if nn:
        keepflag = torch.ones(nn, dtype=torch.int32, device=dev)
        cs = torch.zeros(nn, dtype=torch.float64, device=dev)
        sn = torch.zeros(nn, dtype=torch.float64, device=dev)
        rot = torch.zeros(nn, dtype=torch.int32, device=dev)
        if dev.type == "cuda":
            _hip().stedc_runs(nn, c.data_ptr(), dd.data_ptr(), z.data_ptr(), ty.data_ptr(), tolf, cs.data_ptr(),
                              sn.data_ptr(), rot.data_ptr(), keepflag.data_ptr(),
                              torch.cuda.current_stream(dev).cuda_stream)
        else:
            _runs_host(c, dd, z, ty, tolf, cs, sn, rot, keepflag)
        hb = torch.cat([z, rot.to(torch.float64), keepflag.to(torch.float64),
                        ty.to(torch.float64)]).cpu().numpy()                # host sync 2
        z2_h, rot_h, keep_h = hb[:s], hb[s:s + nn], hb[s + nn:s + 2 * nn]
        ty_h = hb[s + 2 * nn:].astype(np.int64)
        ridx_h = np.nonzero(rot_h)[0]
        if ridx_h.size and nr:
            I, J = _upload(c_h[ridx_h - 1], dev), _upload(c_h[ridx_h], dev)
            rsel = _upload(ridx_h, dev)
            C, S = cs[rsel].contiguous(), sn[rsel].contiguous()
            if dev.type == "cuda":
                _hip().rot_cols(nr, Qs.data_ptr(), max(1, Qs.stride(1)), ridx_h.size, I.data_ptr(), J.data_ptr(),
                                C.data_ptr(), S.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
            else:
                for t in range(ridx_h.size):
                    ii, jj, cc, ss = int(I[t]), int(J[t]), float(C[t]), float(S[t])
                    qi, qj = Qs[:, ii].clone(), Qs[:, jj].clone()
                    Qs[:, ii] = cc * qi - ss * qj
                    Qs[:, jj] = ss * qi + cc * qj
        K_h = c_h[keep_h != 0]
    K = _upload(K_h, dev)
    k = K_h.size
    lam = dd.clone()
    if k:
        dK, zK = dd[K].contiguous(), z[K].contiguous()
        org = torch.empty(k, dtype=torch.int64, device=dev)
        mu = torch.empty(k, dtype=torch.float64, device=dev)
        zh = torch.empty(k, dtype=torch.float64, device=dev)
        if dev.type == "cuda":
            st = torch.cuda.current_stream(dev).cuda_stream
            zzK = float(np.dot(z2_h[K_h], z2_h[K_h]))
            _hip().stedc_secular(k, dK.data_ptr(), zK.data_ptr(), rho, zzK, org.data_ptr(),
                                 mu.data_ptr(), zh.data_ptr(), 0, 0, st)
        else:
            from .eig import stedc_secular as _sec
            _, org_h, mu_h = _sec(dK, zK, rho)
            org.copy_(org_h)
            mu.copy_(mu_h)
            dorg = dK[org]
            delta = (dorg[None, :] - dK[:, None]) + mu[None, :]
            dij = dK[None, :] - dK[:, None]
            ratio = delta / torch.where(dij == 0, torch.ones_like(dij), dij)
            ratio.fill_diagonal_(1.0)
            zh2 = torch.diagonal(delta).clone() * torch.prod(ratio, dim=1) / rho
            zh.copy_(torch.sign(zK) * zh2.abs().sqrt())
        lam[K] = dK[org] + mu
        if nr:
            _merge_gemm(Qs, K, ty_h[K_h], dK, zh, org, mu, lo, m, hi, dev)
    if flip:
        lam = -lam
    o2 = torch.argsort(lam, stable=True)
    w[a:b] = lam[o2]
    if nr:
        Q[lo - r0:hi - r0, a:b] = Qs[:, o2]


def _merge_gemm(Qs, K, tyK_h, dK, zh, org, mu, lo, m, hi, dev):
    """Qs[:, K] <- Qs[:, K] V, V the k x k rank-one vectors (normalised),
    formed CHUNK columns at a time; the rows above m multiply only the K
    columns nonzero there (type 1 or 3), the rows below only type 2 or 3
    (tyK_h: the K columns' types, host)."""
    k = K.numel()
    parts = []
    if lo < m:
        parts.append((0, min(hi, m) - lo, _upload(np.nonzero(tyK_h & 1)[0], dev)))
    if hi > m:
        parts.append((max(lo, m) - lo, hi - lo, _upload(np.nonzero(tyK_h & 2)[0], dev)))
    srcs = []
    for (ra, rb, sel) in parts:
        if sel.numel() == 0:
            srcs.append(None)
            continue
        Ap = ops.colmajor_empty(rb - ra, sel.numel(), torch.float64, dev)
        Ap.copy_(Qs[ra:rb, K[sel]])
        srcs.append(Ap)
    Kd = K
    for j0 in range(0, k, CHUNK):
        nc = min(CHUNK, k - j0)
        V = ops.colmajor_empty(k, nc, torch.float64, dev)
        if dev.type == "cuda":
            _hip().stedc_vectors(k, dK.data_ptr(), zh.data_ptr(), org.data_ptr(), mu.data_ptr(), j0, nc,
                                 V.data_ptr(), max(1, V.stride(1)), torch.cuda.current_stream(dev).cuda_stream)
        else:
            dorg = dK[org[j0:j0 + nc]]
            delta = (dorg[None, :] - dK[:, None]) + mu[None, j0:j0 + nc]
            Vs = zh[:, None] / (-delta)
            V.copy_(Vs / Vs.norm(dim=0, keepdim=True))
        cols = Kd[j0:j0 + nc]
        for (ra, rb, sel), Ap in zip(parts, srcs):
            out = ops.colmajor_zeros(rb - ra, nc, torch.float64, dev)
            if Ap is not None:
                Vp = ops.colmajor_empty(sel.numel(), nc, torch.float64, dev)
                Vp.copy_(V[sel])
                ops.gemm(1.0, Ap, Vp, 0.0, out)
            Qs[ra:rb, cols] = out


def _upload(idx, dev):
    """Host index array -> int64 tensor on dev (pinned, stream-ordered: no
    host synchronisation)."""
    t = torch.from_numpy(np.ascontiguousarray(idx, dtype=np.int64))
    if dev.type != "cuda":
        return t
    return t.pin_memory().to(dev, non_blocking=True)


def _runs_host(c, dd, z, ty, tol, cs, sn, rot, keep):
    """CPU form of stedc_runs_kernel (same arithmetic)."""
    cl = c.tolist()
    dl = dd.tolist()
    nn = len(cl)
    t = 0
    while t < nn:
        acc = float(z[cl[t]])
        tacc = int(ty[cl[t]])
        u = t + 1
        rot[t] = 0
        while u < nn and dl[cl[u]] - dl[cl[u - 1]] <= tol:
            b = float(z[cl[u]])
            r = float(np.hypot(acc, b))
            cs[u] = 1.0 if r == 0 else b / r
            sn[u] = 0.0 if r == 0 else acc / r
            rot[u] = 1
            z[cl[u - 1]] = 0.0
            z[cl[u]] = r
            tacc |= int(ty[cl[u]])
            ty[cl[u]] = tacc
            keep[u - 1] = 0
            acc = r
            u += 1
        keep[u - 1] = 1
        t = u


def stedc(d, e, device=None, leaf=None):
    """One process: (ascending eigenvalues on the host, n x n eigenvectors
    on ``device``)."""
    w, Q, _, _, _ = stedc_rows(d, e, None, device, leaf)
    return w, Q


def stedc_matrix(d, e, comm, device, nb, dtype=torch.float64):
    """Distributed: the eigenvalues and the eigenvector matrix as a
    slate_amd Matrix with one block of rows per rank (p = P, q = 1, row tile
    = the row block, column tile nb) -- ready for redistribute()."""
    from ..core.matrix import Matrix
    w, Q, r0, r1, mb = stedc_rows(d, e, comm, device)
    n = w.numel()
    P = comm.size
    Zr = Matrix(n, n, nb=nb, mb=mb, p=P, q=1, comm=comm, dtype=dtype, device=Q.device)
    Zr.insertLocalTiles(device=Q.device if Q.is_cuda else -1)
    lb = Zr.local_block()
    if lb.mloc != r1 - r0 or lb.nloc != n:
        raise SlateError(f"stedc_matrix: local block {lb.mloc} x {lb.nloc} != {r1 - r0} x {n}")
    if lb.mloc:
        lb.data[:, :].copy_(Q.to(dtype))
    Zr.storage.mark_local_modified(Zr.storage.origin_slot)
    return w, Zr
