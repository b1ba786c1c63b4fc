"""Singular value decomposition: svd (ge2tb -> tb2bd -> bdsqr ->
back-transforms) and its stages ge2tb, tb2bd, bdsqr, unmbr_ge2tb,
unmbr_tb2bd.

Reference: `src/svd.cc:155-364` (optional QR/LQ pre-step, ge2tb, gather
band, tb2bd on the host, bdsqr, back-transforms), `src/ge2tb.cc`,
`src/tb2bd.cc`, `src/bdsqr.cc`, `src/unmbr_ge2tb.cc`, `src/unmbr_tb2bd.cc`.

MI355X design: stage 1 on one GPU (column-panel QR and row-panel LQ by the
recursive GPU QR, two-sided block-reflector updates as MFMA GEMMs), stage 2
and the bidiagonal QR on the host (native C++, like SLATE), back-transforms
on the GPU (one launch per bulge-chasing sweep; GEMM-blocked WY for
stage 1).  Multi-rank (and SLATE_AMD_SVD_DIST=1): the distributed path of
svd_dist.py (ge2tb on the grid, band reduced to rank 0 for tb2bd, bdsqr on
each rank's own rows, back-transforms on the grid).
"""
from __future__ import annotations

import torch

from .. import _native, ops
from ..core.exceptions import SlateError
from ..core.options import get_option
from ..core.enums import Option
from ..utils.trace import trace_block
from ._util import conj_trans
from .eig import _cm, _code, _my_cols, _zero_strict_lower
from .qr import _apply_qh, _vh


class Ge2tbFactors:
    def __init__(self):
        self.left = []     # (row0, V, T): Q_k acting on rows row0..
        self.right = []    # (col0, V, T): P_k acting on columns col0..


def ge2tb(A: torch.Tensor, nb: int):
    """Dense m x n (m >= n, column-major) -> upper band (bandwidth nb) in
    place: A = Ql B Qr^H."""
    m, n = A.shape
    F = Ge2tbFactors()
    ct = conj_trans(A.dtype)
    with trace_block("ge2tb"):
        for k0 in range(0, n, nb):
            kb = min(nb, n - k0)
            P = A[k0:, k0:k0 + kb]
            kk = min(m - k0, kb)
            tau = torch.zeros(kk, dtype=A.dtype, device=A.device)
            T, V = ops.geqrf(P, tau)
            F.left.append((k0, V, T))
            if k0 + kb < n:
                _apply_qh(V, T, A[k0:, k0 + kb:], conj=True, Vh=_vh(V))
            _zero_strict_lower(P)
            c0 = k0 + kb
            if c0 >= n:
                continue
            X = A[k0:k0 + kb, c0:]                                # kb x w
            Xh = _cm(X.mH.contiguous())
            w = Xh.shape[0]
            kr = min(w, kb)
            taur = torch.zeros(kr, dtype=A.dtype, device=A.device)
            Tr, Vr = ops.geqrf(Xh, taur)
            _zero_strict_lower(Xh)
            X.copy_(Xh.mH)
            F.right.append((c0, Vr, Tr))
            C = A[k0 + kb:, c0:]
            if C.shape[0]:
                W = ops.colmajor_empty(C.shape[0], kr, A.dtype, A.device)
                ops.gemm(1.0, C, Vr, 0.0, W)                      # W = C V
                ops.trmm('R', 'U', 'N', 'N', 1.0, Tr, W)          # W = C V T
                ops.gemm(-1.0, W, Vr, 1.0, C, transB=ct)          # C -= W V^H
    return F


class Tb2bdFactors:
    def __init__(self, U, V, pu, pv):
        self.U, self.V, self.pu, self.pv = U, V, pu, pv


def _tb2bd_schedule(n, b):
    """Tasks per sweep of the bidiagonal chase (one right + one left
    reflector each) and the first reflector slot of every sweep."""
    j = torch.arange(max(n - 1, 0), dtype=torch.int64)
    ce0 = torch.clamp(j + b, max=n - 1)
    nt = 1 + torch.div(n - 1 - ce0 + b - 1, b, rounding_mode="floor")
    sp = torch.zeros(max(n, 1), dtype=torch.int64)
    if n > 1:
        sp[1:n] = torch.cumsum(nt, 0)
    return nt, sp


def _tb2bd_device(B: torch.Tensor, b: int, dev):
    """Bidiagonal bulge chasing on the GPU (csrc/hip/hb2st.hip tb2bd_kernel):
    persistent workgroups take sweeps from an atomic ticket, progress
    counters between consecutive sweeps (lag 8), reflectors in the host
    pipeline's slots."""
    n = B.shape[0]
    dt = B.dtype
    ldp = -(-n // 8) * 8 + 72                  # leading dimension off powers of two
    A = torch.empty((n, ldp), dtype=dt, device=dev).t()[:n]
    A.copy_(B.to(dev))
    nt, sp = _tb2bd_schedule(n, b)
    total = int(nt.sum()) if nt.numel() else 0
    cap = max(total, 1)

    def store():
        return (torch.zeros(cap, b, dtype=dt, device=dev), torch.zeros(cap, dtype=dt, device=dev),
                torch.zeros(cap, dtype=torch.int64, device=dev), torch.zeros(cap, dtype=torch.int64, device=dev))
    U = store()
    V = store()
    nsw = max(n - 1, 0)
    work = torch.zeros(nsw + 2, dtype=torch.int32, device=dev)
    ntd, spd = nt.to(dev), sp.to(dev)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    nt0 = int(nt[0]) if nt.numel() else 1
    nwg = int(min(max(nsw, 1), cus, max(8, nt0 // 4 + 8)))
    with trace_block("tb2bd"):
        if nsw > 0:
            _native._hip.tb2bd(_code(dt), n, b, A.data_ptr(), A.stride(1), *(x.data_ptr() for x in U),
                               *(x.data_ptr() for x in V), spd.data_ptr(), ntd.data_ptr(), work.data_ptr(), nsw, nwg,
                               torch.cuda.current_stream(dev).cuda_stream)
    return A, U, V, sp, total


def tb2bd(B: torch.Tensor, nb: int):
    """Upper band (dense copy, bandwidth nb) -> real bidiagonal (d, e) plus
    reflectors and phases.  On the GPU when B is there (bandwidth <= 128;
    SLATE_AMD_TB2BD=host forces the pipelined host threads)."""
    import os
    n = B.shape[0]
    b = max(1, nb)
    if B.is_cuda and b <= 128 and os.environ.get("SLATE_AMD_TB2BD", "device") != "host":
        Ad, (UV, Ut, Ur, Ul), (VV, Vt, Vr, Vl), up, cu = _tb2bd_device(B, b, B.device)
        cv = cu
        vp = up
        dt = Ad.dtype
        dc = Ad.diagonal().cpu().clone()
        ec = Ad.diagonal(1).cpu().clone()
    else:
        Bh = _cm(B.detach().to("cpu").clone())
        Bh = _cm(Bh)
        cap = n * (n // b + 2) + 1
        dt = Bh.dtype

        def store():
            return (torch.zeros(cap, b, dtype=dt), torch.zeros(cap, dtype=dt), torch.zeros(cap, dtype=torch.int64),
                    torch.zeros(cap, dtype=torch.int64))
        UV, Ut, Ur, Ul = store()
        VV, Vt, Vr, Vl = store()
        up = torch.zeros(max(n, 1), dtype=torch.int64)
        vp = torch.zeros(max(n, 1), dtype=torch.int64)
        with trace_block("tb2bd"):
            cu, cv = _native._host.tb2bd(_code(dt), n, b, Bh.data_ptr(), max(1, Bh.stride(1)), UV.data_ptr(),
                                         Ut.data_ptr(), Ur.data_ptr(), Ul.data_ptr(), VV.data_ptr(), Vt.data_ptr(),
                                         Vr.data_ptr(), Vl.data_ptr(), cap, up.data_ptr(), vp.data_ptr())
        dc = Bh.diagonal().clone()
        ec = Bh.diagonal(1).clone()
    d = torch.zeros(n, dtype=torch.float64)
    e = torch.zeros(max(n - 1, 0), dtype=torch.float64)
    pu = torch.ones(n, dtype=dt)
    pv = torch.ones(n, dtype=dt)
    if dt.is_complex:
        dcl, ecl = dc.tolist(), ec.tolist()
        pul, pvl = [1 + 0j] * n, [1 + 0j] * n
        dl, el = [0.0] * n, [0.0] * max(n - 1, 0)
        for i in range(n):
            x = dcl[i] * pvl[i]
            ax = abs(x)
            pul[i] = x / ax if ax > 0 else 1 + 0j
            dl[i] = ax
            if i < n - 1:
                y = pul[i].conjugate() * ecl[i]
                ay = abs(y)
                pvl[i + 1] = (y / ay).conjugate() if ay > 0 else 1 + 0j
                el[i] = ay
        pu = torch.tensor(pul, dtype=dt)
        pv = torch.tensor(pvl, dtype=dt)
        d = torch.tensor(dl, dtype=torch.float64)
        e = torch.tensor(el, dtype=torch.float64)
    else:
        d = dc.to(torch.float64)
        e = ec.to(torch.float64)
    from .eig import Hb2stFactors
    FU = Hb2stFactors(UV[:cu], Ut[:cu], Ur[:cu], Ul[:cu], up, cu, None)
    FV = Hb2stFactors(VV[:cv], Vt[:cv], Vr[:cv], Vl[:cv], vp, cv, None)
    return d, e, Tb2bdFactors(FU, FV, pu, pv)


def bdsqr(d: torch.Tensor, e: torch.Tensor, want_u=True, want_vt=True):
    """SVD of the real upper bidiagonal (d, e): returns (s desc, U, VT)."""
    n = d.numel()
    d = d.to(torch.float64).cpu().clone()
    e = e.to(torch.float64).cpu().clone() if n > 1 else torch.zeros(1, dtype=torch.float64)
    U = _cm(torch.eye(n, dtype=torch.float64)) if want_u else None
    VT = _cm(torch.eye(n, dtype=torch.float64)) if want_vt else None
    with trace_block("bdsqr"):
        f = _native._host.bdsqr(n, d.data_ptr(), e.data_ptr(), U.data_ptr() if U is not None else 0,
                                max(1, n), n if U is not None else 0, VT.data_ptr() if VT is not None else 0,
                                max(1, n), n if VT is not None else 0)
    if f:
        raise SlateError("bdsqr: no convergence")
    return d, U, VT


def unmbr_ge2tb(side, F: Ge2tbFactors, Z: torch.Tensor):
    """Back-transform of stage 1 (src/unmbr_ge2tb.cc): side 'L' applies
    Z := Q Z with Q the product of ge2tb's column-panel reflectors (A = Q B
    P^H), side 'R' applies Z := P Z (the row-panel reflectors; V of the SVD
    is P times the band's V).  Block reflectors, MFMA GEMMs."""
    fac = F.left if str(getattr(side, "value", side))[0] in "Ll" else F.right
    for (r0, V, T) in reversed(fac):
        _apply_qh(V, T, Z[r0:, :], conj=False, Vh=_vh(V))
    return Z


def unmbr_tb2bd(side, F: "Tb2bdFactors", Z: torch.Tensor):
    """Back-transform of stage 2 (src/unmbr_tb2bd.cc): side 'L' applies
    Z := Q_U diag(pu) Z, side 'R' applies Z := Q_V diag(pv) Z, so that the
    band B = Q_U diag(pu) Bd diag(pv)^H Q_V^H with Bd the real bidiagonal
    (on the GPU: one blocked launch over all sweeps, csrc/hip/eig.hip)."""
    left = str(getattr(side, "value", side))[0] in "Ll"
    ph = F.pu if left else F.pv
    Z.mul_(ph.to(Z.device, Z.dtype)[:, None])
    return _unmtr_refl(F.U if left else F.V, Z)


def _unmtr_refl(F, Z):
    from .eig import unmtr_hb2st
    return unmtr_hb2st(F, Z)


def svd(A, S=None, U=None, VH=None, opts=None):
    """Singular values (descending; returned and copied into S) and
    optionally the singular vectors U (m x k) and VH (k x n), k = min(m, n).
    A is destroyed."""
    import os
    from .aux import allgather_dense
    st = A.storage
    if st.bc is not None and (st.comm.size > 1 or os.environ.get("SLATE_AMD_SVD_DIST") == "1"):
        from .svd_dist import svd_dist
        return svd_dist(A, S, U, VH, opts)
    with trace_block("svd"):
        dev = st.device if st.device.type == "cuda" else torch.device("cpu")
        m, n = A.m(), A.n()
        nb = int(get_option(opts, Option.InnerBlocking, 0)) or min(st.bc.nb if st.bc else 64, 128)
        Ad = allgather_dense(A).to(dev)
        trans = m < n
        if trans:
            Ad = Ad.mH
            m, n = n, m
            U, VH = (VH, U)
        Ad = _cm(Ad.contiguous().clone() if not Ad.is_contiguous() else Ad.clone())
        Ad = _cm(Ad)
        amax = Ad.abs().max().item() if Ad.numel() else 0.0
        scale = 1.0
        if amax > 0 and (amax < 1e-140 or amax > 1e140):
            scale = 1.0 / amax
            Ad.mul_(scale)
        F1 = ge2tb(Ad, nb)
        k = n
        # the upper band 0 <= j - i <= nb of the reduced matrix (two masked
        # copies: upper triangle, then rows within nb of the diagonal)
        band = ops.colmajor_empty(k, k, Ad.dtype, Ad.device)
        ops.gecopy_mask(Ad[:k, :k], band, (2, 1 << 40, 1, 0, 1, 0, 0, 0, 0))
        ops.gecopy_mask(band, band, (1, 1 << 40, 1, 0, 1, 0, 0, 0, nb))
        d, e, F2 = tb2bd(band, nb)
        wantU = U is not None
        wantV = VH is not None
        s, Ub, VTb = bdsqr(d, e, wantU, wantV)
        if scale != 1.0:
            s = s / scale
        dt = Ad.dtype
        if wantU:
            Zu = ops.colmajor_zeros(m, k, dt, dev)
            Zu[:k].copy_((F2.pu[:, None] * Ub.to(dt)).to(dev))
            _unmtr_refl(F2.U, Zu[:k])
            for (r0, V, T) in reversed(F1.left):
                _apply_qh(V, T, Zu[r0:, :], conj=False, Vh=_vh(V))
        if wantV:
            Zv = ops.colmajor_empty(k, k, dt, dev)
            Zv.copy_((F2.pv[:, None] * VTb.T.to(dt)).to(dev))
            _unmtr_refl(F2.V, Zv)
            for (c0, V, T) in reversed(F1.right):
                _apply_qh(V, T, Zv[c0:, :], conj=False, Vh=_vh(V))
        # write the outputs: (U, VH) of op(A)
        if trans:
            # A^H = Uu S Vv^H  ->  A = Vv S Uu^H  (U/VH were swapped above:
            # here `U` is the caller's VH and `VH` the caller's U)
            if wantU:
                _store(U, Zu.mH)
            if wantV:
                _store(VH, Zv)
        else:
            if wantU:
                _store(U, Zu)
            if wantV:
                _store(VH, Zv.mH)
        if S is not None:
            S.copy_(s.to(S.dtype).to(S.device)[:S.numel()])
        return s


def _store(M, D):
    from .aux import from_dense
    from_dense(M, D.to(M.storage.device if M.storage.device.type == "cuda" else "cpu"))


def svd_vals(A, S=None, opts=None):
    return svd(A, S, None, None, opts)
