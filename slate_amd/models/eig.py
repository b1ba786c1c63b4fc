"""Hermitian eigensolvers: heev (2-stage), hegst, hegv, and the stage
components he2hb, hb2st, sterf, steqr, stedc, unmtr_he2hb, unmtr_hb2st.

Reference: `src/heev.cc:66-225` (scale -> he2hb -> gather band -> hb2st ->
sterf/steqr/stedc -> back-transforms), `src/he2hb.cc` (panel QR + two-sided
trailing update, square grid required), `src/hb2st.cc` (bulge chasing on
rank 0, multithreaded host), `src/unmtr_he2hb.cc`, `src/unmtr_hb2st.cc`,
`src/stedc*.cc`, `src/steqr.cc`, `src/sterf.cc`, `src/hegst.cc`,
`src/hegv.cc`.

MI355X design:
* stage 1 (he2hb, 4/3 n^3 flops) runs on ONE GPU on the full Hermitian
  matrix (288 GB HBM holds n = 100k+): the panel is the GPU recursive QR,
  the two-sided update is three MFMA GEMMs (Y = A V T, W = Y - V M/2,
  A -= V W^H + W V^H) -- no hemm-on-host split like SLATE's he2hb_hemm;
* stage 2 (hb2st, O(n^2 b)) is a native C++ bulge chase on the host (like
  SLATE), recording every reflector;
* tridiagonal: sterf / steqr (native C++, rotations applied row-parallel)
  or divide & conquer (stedc: secular equations in C++, the eigenvector
  merges are GEMMs on the GPU);
* back-transforms on the GPU: unmtr_hb2st applies one whole sweep of
  (disjoint) reflectors per launch; unmtr_he2hb is the blocked-WY GEMM
  update per panel.
Multi-rank: `eig_dist.heev_dist` -- stage 1 on the process grid, the
band reduced to rank 0 for stage 2, back-transforms on the grid; no rank
holds the dense matrix.
"""
from __future__ import annotations

import contextlib
import os

import torch

from .. import _native, ops
from ..core.enums import MethodEig, Option, Uplo
from ..core.exceptions import SlateError
from ..core.options import get_option
from ..utils.trace import trace_block
from ._util import conj_trans

# ------------------------------------------------------------------ helpers


def _code(dt):
    return {torch.float32: 's', torch.float64: 'd', torch.complex64: 'c', torch.complex128: 'z'}[dt]


def _cm(t):
    return t.t().contiguous().t() if t.dim() == 2 and not (t.stride(0) == 1) else t


def _dense_hermitian(A):
    """Full Hermitian (both triangles) dense copy of a Hermitian matrix."""
    from .aux import allgather_dense
    D = allgather_dense(A)
    up = A.uploPhysical()
    if up in (Uplo.Lower, Uplo.Upper) and D.dim() == 2 and D.shape[0] == D.shape[1]:
        # stored triangle (real diagonal) + the strict opposite triangle of
        # D^H: four slate kernels, no torch compute on the device
        n = D.shape[0]
        D = _cm(D)
        keep = 1 if up == Uplo.Lower else 2
        H = ops.colmajor_empty(n, n, D.dtype, D.device)
        T = ops.colmajor_empty(n, n, D.dtype, D.device)
        ops.gecopy_mask(D, H, (keep, 1 << 40, 1, 0, 1, 0, 0, 0, 0), real_diag=True)
        ops.gecopy(D, T, trans=conj_trans(D.dtype))
        ops.gecopy_mask(T, T, (3 - keep, 1 << 40, 1, 0, 1, 0, 0, 0, -1))
        ops.geadd(1.0, T, 1.0, H)
        return H
    if up == Uplo.Lower:
        L = torch.tril(D)
    elif up == Uplo.Upper:
        L = torch.triu(D).mH
    else:
        return D
    H = L + torch.tril(L, -1).mH
    if H.is_complex():          # Hermitian: imaginary part of the diagonal is ignored (LAPACK)
        H.diagonal().imag.zero_()
    return H


class He2hbFactors:
    """Panel reflectors of stage 1: per panel k the explicit V (rows
    (k+1)nb..n) and T."""

    def __init__(self, nb):
        self.nb = nb
        self.panels = []


# ------------------------------------------------------------------ stage 1
def he2hb(Af: torch.Tensor, nb: int):
    """Reduce the dense Hermitian Af (n x n, column-major, both triangles)
    in place to Hermitian band form (bandwidth nb); returns He2hbFactors.

    On a GPU the panels are pipelined one step ahead (SLATE overlaps them
    with OpenMP tasks, src/he2hb.cc:172-610): the update stream applies the
    rank-2kk update of step k to the NEXT panel's columns first, the panel
    stream then QR-factors that panel while the update stream streams the
    rest of the trailing matrix.  The rows of the next panel's band block
    (A22[0:nb, nb:]) are skipped by that bulk GEMM: the next step overwrites
    them with R^H, and nothing reads them before."""
    n = Af.shape[0]
    F = He2hbFactors(nb)
    ct = conj_trans(Af.dtype)
    from ..parallel.streams import StreamSet
    pipe = Af.is_cuda and os.environ.get("SLATE_AMD_HE2HB_PIPE", "1") != "0"
    ss = StreamSet(Af.device, reserve_cus=0) if pipe else None   # GEMM-shaped QR panel: no reserved CUs
    ev_cols = None                      # step k-1's update of this step's panel columns
    with trace_block("he2hb"):
        if pipe:
            ss.fork(diag=False)
        for k0 in range(0, max(n - nb, 0), nb):
            r0 = k0 + nb
            kb = min(nb, n - k0)
            m = n - r0
            if m <= 0:
                break
            kk = min(m, kb)
            with (ss.use(ss.panel) if pipe else contextlib.nullcontext()):
                if pipe and ev_cols is not None:
                    ss.wait(ss.panel, ev_cols)
                P = Af[r0:, k0:k0 + kb]
                tau = torch.zeros(kk, dtype=Af.dtype, device=Af.device)
                T, V = ops.geqrf(P, tau)
                F.panels.append((r0, V, T))
                # band part: keep R, zero the reflectors, mirror to the upper triangle
                _zero_strict_lower(P)
                Af[k0:k0 + kb, r0:].copy_(P.mH)
                X = ops.colmajor_empty(m, kk, Af.dtype, Af.device)
                X.copy_(V)
                ops.trmm('R', 'U', 'N', 'N', 1.0, T, X)                 # X = V T
                ev_qr = ss.event(ss.panel) if pipe else None
            us = ss.update[0] if pipe else None
            with (ss.use(us) if pipe else contextlib.nullcontext()):
                if pipe:
                    ss.wait(us, ev_qr)
                    for t_ in (V, T, X):
                        t_.record_stream(us)
                # two-sided update of the trailing matrix
                A22 = Af[r0:, r0:]
                # [V W] and [W V] side by side: the rank-2kk update A -= V W^H +
                # W V^H is ONE GEMM with K = 2 kk (A22 streamed once, not twice)
                VW = ops.colmajor_empty(m, 2 * kk, Af.dtype, Af.device)
                WV = ops.colmajor_empty(m, 2 * kk, Af.dtype, Af.device)
                Y = VW[:, kk:]
                ops.gemm(1.0, A22, X, 0.0, Y)                            # Y = A V T
                Mt = ops.colmajor_empty(kk, kk, Af.dtype, Af.device)
                ops.gemm(1.0, X, Y, 0.0, Mt, transA=ct)                  # M = T^H V^H Y
                ops.gemm(-0.5, V, Mt, 1.0, Y)                            # W = Y - V M / 2
                VW[:, :kk].copy_(V)
                WV[:, :kk].copy_(Y)
                WV[:, kk:].copy_(V)
                nxt = min(nb, m) if pipe and m > nb else 0
                if nxt:
                    # the next panel's columns first (all rows), then the rest
                    # below the next band block
                    ops.gemm(-1.0, VW, WV[:nxt], 1.0, A22[:, :nxt], transB=ct)
                    ev_cols = ss.event(us)
                    ops.gemm(-1.0, VW[nxt:], WV[nxt:], 1.0, A22[nxt:, nxt:], transB=ct)
                else:
                    ops.gemm(-1.0, VW, WV, 1.0, A22, transB=ct)          # A -= V W^H + W V^H
                    ev_cols = ss.event(us) if pipe else None
        if pipe:
            ss.join()
    return F


def _zero_strict_lower(P):
    """P's strictly lower part set to zero in place (one slate kernel)."""
    m, k = P.shape
    if m > 1 and k:
        ops.gecopy_mask(P, P, (2, 1 << 40, 1, 0, 1, 0, 0, 0, 0))


def unmtr_he2hb(F: He2hbFactors, Z: torch.Tensor):
    """Z := Q1 Z (Q1 = Q_0 Q_1 ... from he2hb): panels applied last-to-first.

    On a GPU, groups of SLATE_AMD_UNMTR_HE2HB_GROUP (default 8) consecutive
    panels are merged into one block reflector I - V T V^H (forward larft
    merge, T = [[T1, -T1 V1^H V2 T2], [0, T2]]): Z is streamed once per
    group with K = 8 nb instead of once per panel with K = nb."""
    with trace_block("unmtr_he2hb"):
        from .qr import _apply_qh, _vh
        groups = getattr(F, "groups", None)
        if groups is not None and Z.is_cuda:
            # built ahead on the side stream (premerge_groups)
            torch.cuda.current_stream(Z.device).wait_event(F.ready)
            for r0, Vg, Tg, Vh in groups:
                _apply_qh(Vg, Tg, Z[r0:, :], conj=False, Vh=Vh)
            return Z
        panels = F.panels
        grp = _he2hb_group(Z.is_cuda)
        i1 = len(panels)
        while i1 > 0:
            i0 = max(0, i1 - grp)
            if i1 - i0 == 1:
                r0, V, T = panels[i0]
                _apply_qh(V, T, Z[r0:, :], conj=False, Vh=_vh(V))
            else:
                r0, Vg, Tg = _merge_reflectors(panels[i0:i1])
                _apply_qh(Vg, Tg, Z[r0:, :], conj=False, Vh=_vh(Vg))
            i1 = i0
    return Z


def _he2hb_group(gpu):
    # 8 panels per block reflector on a GPU: dsyevd n = 16384 1.995 s (4) ->
    # 1.984 s (8), profiles/r6/heev/py_group_4_vs_8.txt
    return max(1, int(os.environ.get("SLATE_AMD_UNMTR_HE2HB_GROUP", "8" if gpu else "1")))


def premerge_groups(F: He2hbFactors, device):
    """Build unmtr_he2hb's merged block reflectors (and their explicit V^H)
    on the pipeline's panel stream, right after he2hb: they then run while
    the bulge chase holds ~100 of the 256 CUs instead of after it.
    unmtr_he2hb waits for F.ready before applying them.  No-op off the GPU,
    on a serial stream set or with SLATE_AMD_HEEV_OVERLAP=0."""
    if device.type != "cuda" or os.environ.get("SLATE_AMD_HEEV_OVERLAP", "1") == "0":
        return
    from ..parallel.streams import StreamSet
    from .qr import _vh
    ss = StreamSet(device, reserve_cus=0)
    main = torch.cuda.current_stream(device)
    side = ss.panel
    if side is None or side == main:
        return
    side.wait_event(ss.event(main))
    panels, grp, out = F.panels, _he2hb_group(True), []
    with torch.cuda.stream(side):
        for _, V, T in panels:
            V.record_stream(side)
            T.record_stream(side)
        i1 = len(panels)
        while i1 > 0:
            i0 = max(0, i1 - grp)
            if i1 - i0 == 1:
                r0, Vg, Tg = panels[i0]
            else:
                r0, Vg, Tg = _merge_reflectors(panels[i0:i1])
            Vh = _vh(Vg)
            for t in (Vg, Tg, Vh):
                if t is not None:
                    t.record_stream(main)
            out.append((r0, Vg, Tg, Vh))
            i1 = i0
    F.groups = out
    F.ready = ss.event(side)


def _merge_reflectors(group):
    """One block reflector for the product H_0 H_1 ... of consecutive panel
    reflectors (r_i, V_i, T_i) (V_i explicit, rows r_i..n-1; T_i upper)."""
    ct = None
    r0 = group[0][0]
    m = group[0][1].shape[0]
    dt, dev = group[0][1].dtype, group[0][1].device
    ct = conj_trans(dt)
    ktot = sum(V.shape[1] for _, V, _ in group)
    Vg = ops.colmajor_zeros(m, ktot, dt, dev)
    Tg = ops.colmajor_zeros(ktot, ktot, dt, dev)
    c = 0
    for (r, V, T) in group:
        kb = V.shape[1]
        off = r - r0
        Vg[off:, c:c + kb].copy_(V)
        ops.gecopy_mask(T[:kb, :kb], Tg[c:c + kb, c:c + kb], (2, 1 << 40, 1, 0, 1, 0, 0, 0, 0))   # triu
        if c:
            # T12 = -T_prev (V_prev^H V_i) T_i over the rows V_i spans
            S = ops.colmajor_empty(c, kb, dt, dev)
            ops.gemm(1.0, Vg[off:, :c], V, 0.0, S, transA=ct)
            S2 = ops.colmajor_empty(c, kb, dt, dev)
            ops.gemm(1.0, S, Tg[c:c + kb, c:c + kb], 0.0, S2)
            ops.gemm(-1.0, Tg[:c, :c], S2, 0.0, Tg[:c, c:c + kb])
        c += kb
    return r0, Vg, Tg


# ------------------------------------------------------------------ stage 2
class Hb2stFactors:
    def __init__(self, V, tau, row, length, sweep_ptr, count, phase):
        self.V, self.tau, self.row, self.length = V, tau, row, length
        self.sweep_ptr, self.count, self.phase = sweep_ptr, count, phase


def _hb2st_schedule(n, b):
    """Tasks per sweep (same recurrence as the chase) and the first
    reflector slot of every sweep."""
    j = torch.arange(max(n - 1, 0), dtype=torch.int64)
    e0 = torch.clamp(j + b, max=n - 1)
    k0 = e0 - j
    nt = torch.where(k0 <= 1, torch.zeros_like(j), 1 + torch.div(n - 1 - e0 + b - 1, b, rounding_mode="floor"))
    sp = torch.zeros(max(n, 1), dtype=torch.int64)
    if n > 1:
        sp[1:n] = torch.cumsum(nt, 0)
    return nt, sp


_HB2ST_PROF = {}     # tools: {"buf": int64 device tensor(5)} -> per-phase clock totals


def _hb2st_device(B: torch.Tensor, nb: int, dev):
    """Bulge chasing on the GPU (csrc/hip/hb2st.hip): persistent
    workgroups, one per concurrently chased sweep, ordered by an atomic
    ticket, progress counters between consecutive sweeps."""
    import os
    from .. import _native
    n = B.shape[0]
    b = max(1, nb)
    dt = B.dtype
    # leading dimension off powers of two: the chase touches ~3b columns of
    # one row band at a time, which a 2^k stride would put on one memory
    # channel
    ldp = -(-n // 8) * 8 + 72
    A = torch.empty((n, ldp), dtype=dt, device=dev).t()[:n]
    A.copy_(B.to(dev))
    nt, sp = _hb2st_schedule(n, b)
    total = int(nt.sum()) if nt.numel() else 0
    V = torch.zeros(max(total, 1), b, dtype=dt, device=dev)
    tau = torch.zeros(max(total, 1), dtype=dt, device=dev)
    row = torch.zeros(max(total, 1), dtype=torch.int64, device=dev)
    ln = torch.zeros(max(total, 1), dtype=torch.int64, device=dev)
    nsw = max(n - 1, 0)
    work = torch.zeros(nsw + 2, dtype=torch.int32, device=dev)
    ntd, spd = nt.to(dev), sp.to(dev)
    props = torch.cuda.get_device_properties(dev)
    # sweeps in flight are bounded by (tasks of a sweep) / lag: more
    # workgroups would only poll
    nt0 = int(nt[0]) if nt.numel() else 1
    # = the kernel's (hb2st.hip): early publication keeps sweeps 2 tasks
    # apart, else `lag` tasks
    lag = max(3, int(os.environ.get("SLATE_AMD_HB2ST_LAG", 3)))
    if os.environ.get("SLATE_AMD_HB2ST_EARLY", "1") != "0":
        lag = 2
    # ~nt0 / 3 workgroups: fewer sweeps in flight than the lag allows leave
    # more L2 / memory bandwidth to the ones that are (dsyevd n = 16384,
    # profiles/r4: 100 workgroups 2.089-2.102 s, 136 = nt0 / lag + 8: 2.128-2.148 s)
    nwg = int(min(max(nsw, 1), props.multi_processor_count, max(8, min(nt0 // lag + 8, nt0 // 3 + 15))))
    nwg = int(os.environ.get("SLATE_AMD_HB2ST_WG", nwg))
    with trace_block("hb2st"):
        if nsw > 0:
            prof = _HB2ST_PROF.get("buf")
            _native._hip.hb2st(_code(dt), n, b, A.data_ptr(), A.stride(1), V.data_ptr(), tau.data_ptr(),
                               row.data_ptr(), ln.data_ptr(), spd.data_ptr(), ntd.data_ptr(), work.data_ptr(),
                               nsw, nwg, torch.cuda.current_stream(dev).cuda_stream,
                               prof.data_ptr() if prof is not None else 0)
    Bh = A
    return Bh, V[:total], tau[:total], row[:total], ln[:total], sp, total


def hb2st(B: torch.Tensor, nb: int, device=None):
    """Hermitian band (dense copy, both triangles, bandwidth nb) -> real
    symmetric tridiagonal (d, e) + reflectors.  On the GPU when ``device``
    is a CUDA device (SLATE_AMD_HB2ST=host forces the pipelined host
    threads: 4.6 s vs 2.6 s on the GPU at n = 16384, b = 64)."""
    import os
    if device is not None and torch.device(device).type == "cuda" and \
            os.environ.get("SLATE_AMD_HB2ST", "device") != "host" and max(1, nb) <= 128:
        Bh, V, tau, row, ln, sp, cnt = _hb2st_device(B, nb, torch.device(device))
        return _hb2st_finish(Bh, V, tau, row, ln, sp, cnt)
    n = B.shape[0]
    Bh = _cm(B.detach().to("cpu")).clone()
    Bh = _cm(Bh)
    b = max(1, nb)
    cap = n * (n // b + 2) + 1
    dt = Bh.dtype
    V = torch.zeros(cap, b, dtype=dt)
    tau = torch.zeros(cap, dtype=dt)
    row = torch.zeros(cap, dtype=torch.int64)
    ln = torch.zeros(cap, dtype=torch.int64)
    sp = torch.zeros(max(n, 1), dtype=torch.int64)
    with trace_block("hb2st"):
        cnt = _native._host.hb2st(_code(dt), n, b, Bh.data_ptr(), max(1, Bh.stride(1)), V.data_ptr(),
                                  tau.data_ptr(), row.data_ptr(), ln.data_ptr(), cap, sp.data_ptr())
    return _hb2st_finish(Bh, V, tau, row, ln, sp, cnt)


def _hb2st_finish(Bh, V, tau, row, ln, sp, cnt):
    n = Bh.shape[0]
    dt = Bh.dtype
    d = Bh.diagonal().real.to(torch.float64).cpu().clone()
    ec = Bh.diagonal(-1).cpu().clone()
    ph = torch.ones(n, dtype=dt)
    if dt.is_complex and n > 1:
        a = ec.abs()
        u = torch.where(a > 0, ec / torch.where(a > 0, a, torch.ones_like(a)), torch.ones_like(ec))
        ph[1:] = torch.cumprod(u, 0)
        e = a.to(torch.float64)
    else:
        e = ec.real.to(torch.float64) if dt.is_complex else ec.to(torch.float64)
    return d, e, Hb2stFactors(V[:cnt], tau[:cnt], row[:cnt], ln[:cnt], sp, cnt, ph)


def unmtr_hb2st(F: Hb2stFactors, Z: torch.Tensor):
    """Z := Q2 Phase Z: one launch per sweep, sweeps last-to-first."""
    if F.phase is not None and Z.dtype.is_complex:
        Z.mul_(F.phase.to(Z.device)[:, None])
    dev = Z.device
    V, tau, row, ln = (x.to(dev) for x in (F.V, F.tau, F.row, F.length))
    n = F.sweep_ptr.numel()
    b = V.shape[1] if V.dim() == 2 else 0
    if Z.is_cuda and n > 1 and F.count > 0 and Z.shape[0] == n and \
            os.environ.get("SLATE_AMD_UNMTR_BLOCKED", "1") != "0":
        # all sweeps in one launch, blocks of b sweeps (csrc/hip/eig.hip)
        # the schedule's index arrays on the host (O(n) ints), uploaded once
        import numpy as np
        sph = F.sweep_ptr.cpu().numpy().astype(np.int64)
        nth = (sph[1:] - sph[:-1]).astype(np.int64)
        up = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.int64)).to(dev)
        spd, ntd = up(sph), up(nth)
        if Z.dtype == torch.float64 and b == 64 and os.environ.get("SLATE_AMD_UNMTR_MFMA", "1") != "0":
            # groups of b reflectors as block reflectors I - V T V^H on MFMA:
            # group g = (block J, task t); T of every group built once
            nsw = n - 1
            TJh = nth[::b]
            ng = int(TJh.sum())
            gJh = np.repeat(np.arange(TJh.size, dtype=np.int64), TJh)
            gptrh = np.zeros(TJh.size + 1, dtype=np.int64)
            gptrh[1:] = np.cumsum(TJh)
            gth = np.arange(ng, dtype=np.int64) - gptrh[gJh]
            gJ, gptr, gt = up(gJh), up(gptrh), up(gth)
            Tg = torch.empty(max(ng, 1) * 2 * b * b, dtype=torch.float64, device=dev)   # Y = V T per group
            with trace_block("unmtr_hb2st"):
                _native.hip().unmtr_hb2st_mfma(n, Z.shape[1], Z.data_ptr(), max(1, Z.stride(1)),
                                               V.contiguous().data_ptr(), b, tau.contiguous().data_ptr(),
                                               spd.data_ptr(), ntd.data_ptr(), gJ.data_ptr(), gt.data_ptr(),
                                               gptr.data_ptr(), ng, Tg.data_ptr(), nsw,
                                               torch.cuda.current_stream(dev).cuda_stream)
            return Z
        with trace_block("unmtr_hb2st"):
            if _native.hip().unmtr_hb2st_blocked(_code(Z.dtype), n, Z.shape[1], Z.data_ptr(), max(1, Z.stride(1)),
                                                 V.contiguous().data_ptr(), b, tau.contiguous().data_ptr(),
                                                 spd.data_ptr(), ntd.data_ptr(), n - 1, False,
                                                 torch.cuda.current_stream(dev).cuda_stream):
                return Z
    sp = F.sweep_ptr.tolist()
    with trace_block("unmtr_hb2st"):
        for j in range(n - 1, -1, -1):
            first = sp[j]
            last = sp[j + 1] if j + 1 < n else F.count
            if last > first:
                ops.apply_refl(Z, V, tau, row, ln, first, last - first)
    return Z


# ------------------------------------------------------------------ tridiagonal
def sterf(d: torch.Tensor, e: torch.Tensor) -> torch.Tensor:
    """Eigenvalues of the symmetric tridiagonal (d, e), ascending."""
    d = d.to(torch.float64).cpu().clone()
    e = e.to(torch.float64).cpu().clone()
    n = d.numel()
    if n and _native._host.sterf(n, d.data_ptr(), e.data_ptr() if n > 1 else d.data_ptr()):
        raise SlateError("sterf: no convergence")
    return d


def steqr(d: torch.Tensor, e: torch.Tensor, Z0=None):
    """Eigenvalues + vectors of the tridiagonal; Z0 (n x k host) is
    rotated as Z0 Q (default: identity -> Q)."""
    d = d.to(torch.float64).cpu().clone()
    e = e.to(torch.float64).cpu().clone()
    n = d.numel()
    Z = torch.eye(n, dtype=torch.float64) if Z0 is None else Z0.to(torch.float64).cpu().clone()
    Z = _cm(Z)
    if n:
        f = _native._host.steqr(n, d.data_ptr(), e.data_ptr() if n > 1 else d.data_ptr(), Z.data_ptr(),
                                max(1, Z.stride(1)), Z.shape[0])
        if f:
            raise SlateError("steqr: no convergence")
    return d, Z


def stedc(d: torch.Tensor, e: torch.Tensor, device=None, leaf=None):
    """Divide & conquer (Cuppen / Gu-Eisenstat) for the symmetric
    tridiagonal (d, e): returns ascending eigenvalues (host fp64) and Z on
    ``device`` (models/stedc.py: GPU leaves, device deflation, split merge
    GEMMs; the distributed form keeps Z row-distributed)."""
    from .stedc import stedc as _stedc
    d = d.to(torch.float64).cpu()
    e = e.to(torch.float64).cpu()
    return _stedc(d.numpy(), e.numpy(), device=device, leaf=leaf)


def _dc(d, e, dev, leaf):
    n = d.numel()
    if n <= leaf:
        w, Z = steqr(d, e)
        return w, Z.to(dev)
    m = n // 2
    rho = float(e[m - 1])
    d1 = d[:m].clone()
    d2 = d[m:].clone()
    d1[-1] -= rho
    d2[0] -= rho
    w1, Q1 = _dc(d1, e[:m - 1], dev, leaf)
    w2, Q2 = _dc(d2, e[m:], dev, leaf)
    z = torch.cat([Q1[-1, :].cpu(), Q2[0, :].cpu()]).to(torch.float64)
    dd = torch.cat([w1, w2])
    Qb = torch.zeros(n, n, dtype=torch.float64, device=dev)
    Qb[:m, :m] = Q1
    Qb[m:, m:] = Q2
    w, U = _rank_one_eig(dd, z, rho, Qb)
    return w, U


def stedc_sort(dd, z, Q):
    """Merge step 1 (src/stedc_sort.cc role): poles ascending, z and the
    columns of Q permuted alike."""
    order = torch.argsort(dd)
    return dd[order].clone(), z[order].clone(), Q[:, order.to(Q.device)].clone()


def stedc_deflate(dd, z, rho, Q):
    """Merge step 2 (src/stedc_deflate.cc): deflate tiny z components and
    (nearly) equal poles; equal poles get a Givens rotation that moves their
    z weight into one of them (the rotation is applied to Q's columns).
    Returns (z, keep): the non-deflated indices in ascending pole order."""
    n = dd.numel()
    eps = torch.finfo(torch.float64).eps
    tol = 8.0 * eps * max(dd.abs().max().item() if n else 0.0, rho * float((z * z).sum()))
    znorm = float(z.norm())
    defl = (rho * z.abs() * znorm <= tol)
    idx = [i for i in range(n) if not defl[i]]
    zl = z.tolist()
    dl = dd.tolist()
    keep, rots = [], []
    prev = None
    for i in idx:
        if prev is not None and abs(dl[i] - dl[prev]) <= tol:
            a, b = zl[prev], zl[i]
            r = (a * a + b * b) ** 0.5
            c, s = b / r, a / r
            rots.append((prev, i, c, s))           # new z_prev = 0, z_i = r
            zl[prev], zl[i] = 0.0, r
            keep[-1] = i
            prev = i
            continue
        keep.append(i)
        prev = i
    for (i, j, c, s) in rots:
        qi, qj = Q[:, i].clone(), Q[:, j].clone()
        Q[:, i] = c * qi - s * qj
        Q[:, j] = s * qi + c * qj
    return torch.tensor(zl, dtype=torch.float64), torch.tensor(keep, dtype=torch.int64)


def stedc_secular(dK, zK, rho):
    """Merge step 3 (src/stedc_secular.cc): roots of the secular equation
    1 + rho sum z_i^2 / (d_i - lambda) = 0 for ascending poles dK (host fp64,
    native C++).  Returns (lambda, org, mu) with lambda_j = dK[org_j] + mu_j
    (the root stored relative to its closest pole, as LAPACK laed4)."""
    k = dK.numel()
    dK = dK.to(torch.float64).contiguous()
    zK = zK.to(torch.float64).contiguous()
    org = torch.zeros(k, dtype=torch.int64)
    mu = torch.zeros(k, dtype=torch.float64)
    if k:
        _native._host.secular(k, dK.data_ptr(), zK.data_ptr(), float(rho), org.data_ptr(), mu.data_ptr())
    return dK[org] + mu, org, mu


def stedc_z_vector(dK, zK, rho, org, mu):
    """Merge step 4 (src/stedc_z_vector.cc role, Gu-Eisenstat): the z_hat
    for which the computed roots are exact, and the normalised eigenvector
    matrix of the rank-one problem, v_j[i] = z_hat_i / (d_i - lambda_j)."""
    dorg = dK[org]
    delta = (dorg[None, :] - dK[:, None]) + mu[None, :]   # lambda_j - d_i, (k x k)
    dij = dK[None, :] - dK[:, None]                        # d_j - d_i
    ratio = delta / torch.where(dij == 0, torch.ones_like(dij), dij)
    ratio.fill_diagonal_(1.0)
    zh2 = torch.diagonal(delta).clone() * torch.prod(ratio, dim=1) / rho
    zh = torch.sign(zK) * zh2.abs().sqrt()
    Vs = zh[:, None] / (-delta)
    return zh, Vs / Vs.norm(dim=0, keepdim=True)


def _rank_one_eig(dd, z, rho, Qb):
    """Eigen-decomposition of Qb (diag(dd) + rho z z^T) Qb^T: returns
    (ascending eigenvalues, Qb @ eigenvectors).  Sort, deflate, secular
    roots, Gu-Eisenstat vectors, one merge GEMM (on the GPU: roots, z_hat
    and the vector matrix by csrc/hip/stedc.hip)."""
    dev = Qb.device
    if rho == 0.0:
        order = torch.argsort(dd)
        return dd[order].clone(), Qb[:, order.to(dev)]
    flip = rho < 0
    if flip:
        dd = -dd
        rho = -rho
    dd, z, Q = stedc_sort(dd, z, Qb)
    z, K = stedc_deflate(dd, z, rho, Q)
    k = K.numel()
    lam = dd.clone()
    if k and dev.type == "cuda":
        dKd = dd[K].contiguous().to(dev)
        zKd = z[K].contiguous().to(dev)
        org = torch.empty(k, dtype=torch.int64, device=dev)
        mu = torch.empty(k, dtype=torch.float64, device=dev)
        zh = torch.empty(k, dtype=torch.float64, device=dev)
        VsC = ops.colmajor_empty(k, k, torch.float64, dev)
        _native.hip().stedc_secular(k, dKd.data_ptr(), zKd.data_ptr(), float(rho), float((z[K] * z[K]).sum()),
                                    org.data_ptr(), mu.data_ptr(), zh.data_ptr(), VsC.data_ptr(), VsC.stride(1),
                                    torch.cuda.current_stream(dev).cuda_stream)
        lam[K] = (dKd[org] + mu).cpu()
    elif k:
        dK, zK = dd[K].contiguous(), z[K].contiguous()
        lamK, org, mu = stedc_secular(dK, zK, rho)
        _, Vs = stedc_z_vector(dK, zK, rho, org, mu)
        lam[K] = lamK
        VsC = ops.as_colmajor(Vs.to(dev))
    if k:
        Kd = K.to(dev)
        QK = ops.as_colmajor(Q[:, Kd])
        Out = ops.colmajor_empty(QK.shape[0], k, Q.dtype, dev)
        ops.gemm(1.0, QK, VsC, 0.0, Out)                 # merge GEMM on the MFMA kernels
        Q[:, Kd] = Out
    if flip:
        lam = -lam
    o2 = torch.argsort(lam)
    return lam[o2].clone(), Q[:, o2.to(dev)].contiguous()


# ------------------------------------------------------------------ drivers
def heev(A, Lambda=None, Z=None, opts=None):
    """Eigenvalues (ascending, returned and copied into Lambda if given) and,
    if Z is given, eigenvectors of the Hermitian matrix A (A is destroyed
    like in SLATE)."""
    import os
    from .aux import from_dense
    s = A.storage
    if s.bc is not None and (s.comm.size > 1 or os.environ.get("SLATE_AMD_EIG_DIST") == "1"):
        from .eig_dist import heev_dist
        return heev_dist(A, Lambda, Z, opts)
    with trace_block("heev"):
        s = A.storage
        dev = s.device if s.device.type == "cuda" else torch.device("cpu")
        # stage-1 band: 64 by default, independent of the tile size (stage 2
        # costs O(n^2 band) on the host; the bulge chase parallelises over
        # n / (4 band) concurrent tasks)
        nb = int(get_option(opts, Option.InnerBlocking, 0)) or min(s.bc.nb if s.bc else 64, 64)
        method = get_option(opts, Option.MethodEig, MethodEig.DC)
        Af = _cm(_dense_hermitian(A).to(dev))
        n = Af.shape[0]
        # scale to a safe range (heev.cc:66-80)
        from ._util import read_to_host
        amax = float(read_to_host(ops.genorm_local('M', Af)[0]).max()) if n else 0.0
        scale = 1.0
        if amax > 0 and (amax < 1e-140 or amax > 1e140):
            scale = 1.0 / amax
            Af.mul_(scale)
        F1 = he2hb(Af, nb)
        if Z is not None:
            premerge_groups(F1, Af.device)
        d, e, F2 = hb2st(_band_only(Af, nb), nb, device=Af.device if Af.is_cuda else None)
        want = Z is not None
        if not want:
            w = sterf(d, e)
        elif method in (MethodEig.QR, 'Q', "qr"):
            w, Zt = steqr(d, e)
        else:
            w, Zt = stedc(d, e, device=dev)
        if scale != 1.0:
            w = w / scale
        if want:
            # back-transform only this rank's columns of Z
            cols = _my_cols(Z)
            if cols == list(range(n)):                # every column local: no gather
                Zl = _cm(Zt.to(dev).to(Af.dtype))
            else:
                Zl = _cm(Zt.to(dev)[:, cols].to(Af.dtype)) if len(cols) else \
                    torch.zeros(n, 0, dtype=Af.dtype, device=dev)
            Zl = _cm(Zl.clone())
            unmtr_hb2st(F2, Zl)
            unmtr_he2hb(F1, Zl)
            _scatter_cols(Z, Zl, cols)
        if Lambda is not None:
            Lambda.copy_(w.to(Lambda.dtype).to(Lambda.device))
        return w


def _band_only(Af, nb):
    """Copy of Af restricted to the band |i - j| <= nb (two masked copies)."""
    n = Af.shape[0]
    B = ops.colmajor_empty(n, n, Af.dtype, Af.device)
    ops.gecopy_mask(Af, B, (2, 1 << 40, 1, 0, 1, 0, 0, 0, nb))        # i <= j + nb
    ops.gecopy_mask(B, B, (1, 1 << 40, 1, 0, 1, 0, 0, 0, nb))         # i + nb >= j
    return B


def _my_cols(Z):
    """Global column indices whose data this rank holds in Z's local block."""
    s = Z.storage
    if s.bc is None:
        return list(range(Z.n()))
    lb = Z.local_block()
    return [lb.global_col(j) for j in range(lb.nloc)]


def _scatter_cols(Z, Zl, cols):
    """Write the n x len(cols) block Zl into this rank's local part of Z."""
    s = Z.storage
    lb = Z.local_block()
    if s.bc is None or lb.mloc == 0 or lb.nloc == 0:
        return
    rows = [lb.global_row(i) for i in range(lb.mloc)]
    if rows == list(range(Zl.shape[0])):
        lb.data.copy_(Zl.to(lb.data.device, lb.data.dtype))           # all rows local: a plain copy
    else:
        lb.data.copy_(Zl[torch.tensor(rows, device=Zl.device)].to(lb.data.device, lb.data.dtype))
    s.mark_local_modified(s.origin_slot)


def eig_vals(A, Lambda=None, opts=None):
    return heev(A, Lambda, None, opts)


def eig(A, Lambda=None, Z=None, opts=None):
    return heev(A, Lambda, Z, opts)


def hegst(itype, A, B, opts=None):
    """Reduce the generalized problem to standard form with the Cholesky
    factor L of B (B = L L^H, from potrf): itype 1: A := L^{-1} A L^{-H};
    itype 2/3: A := L^H A L (src/hegst.cc).  Works on a full-Hermitian
    block-cyclic copy of A with the distributed trsm / trmm (no gather);
    the stored triangle is copied back and the other one is untouched."""
    from .blas3 import trsm, trmm
    from .eig_dist import full_hermitian_copy
    from .aux import copy
    from ..core.matrix import TriangularMatrix
    from ..core.enums import Diag, Side
    with trace_block("hegst"):
        F = full_hermitian_copy(A)
        lower = B.uploPhysical() == Uplo.Lower
        Tb = TriangularMatrix(Uplo.Lower if lower else Uplo.Upper, B, diag=Diag.NonUnit)
        L = Tb if lower else Tb.conj_transpose()          # B = L L^H
        if itype == 1:
            trsm(Side.Left, 1.0, L, F, opts)                     # L^{-1} A
            trsm(Side.Right, 1.0, L.conj_transpose(), F, opts)   # ... L^{-H}
        else:
            trmm(Side.Left, 1.0, L.conj_transpose(), F, opts)    # L^H A
            trmm(Side.Right, 1.0, L, F, opts)                    # ... L
        copy(TriangularMatrix(A.uploPhysical(), F), TriangularMatrix(A.uploPhysical(), A))
    return 0


def _store_tri(R, A):
    up = A.uploPhysical()
    if up == Uplo.Lower:
        return torch.tril(R)
    if up == Uplo.Upper:
        return torch.triu(R)
    return R


def hegv(itype, A, B, Lambda=None, Z=None, opts=None):
    """Generalized Hermitian-definite eigenproblem (src/hegv.cc): potrf(B),
    hegst, heev, back-substitution of the eigenvectors."""
    from .chol import potrf
    from .blas3 import trsm, trmm
    from ..core.matrix import TriangularMatrix
    from ..core.enums import Diag, Side
    with trace_block("hegv"):
        info = potrf(B, opts)
        if info:
            return None
        hegst(itype, A, B, opts)
        w = heev(A, Lambda, Z, opts)
        if Z is not None:
            lower = B.uploPhysical() == Uplo.Lower
            Tb = TriangularMatrix(Uplo.Lower if lower else Uplo.Upper, B, diag=Diag.NonUnit)
            L = Tb if lower else Tb.conj_transpose()          # B = L L^H
            if itype in (1, 2):
                trsm(Side.Left, 1.0, L.conj_transpose(), Z, opts)   # x = L^{-H} y
            else:
                trmm(Side.Left, 1.0, L, Z, opts)                    # x = L y
        return w
