"""Out-of-core Cholesky for a host-resident matrix factored on the GPU.

Reference: the host-origin / device-target workspace streaming of SLATE
(include/slate/BaseMatrix.hh:2640-2781 tileGetForWriting / tileRelease,
3878-3972 releaseWorkspace): tiles travel to the device on demand and are
released after their last use, so a matrix need not fit in device memory.

MI355X design: one rank, the matrix in host memory (origin Host,
Target.Devices), larger than the device budget (or forced with
SLATE_AMD_OOC_COLS).  Left-looking by block columns of W columns:

  for each block column J (rows >= J0 only):
      P  <- A[J0:, J]                              host -> device
      for each finished block column K < J (streamed, double-buffered on a
      copy stream, the next one in flight during the current GEMM):
          P -= L[J0:, K] L[J0:J0+w, K]^H          (one masked MFMA GEMM)
      potrf of P's diagonal block (the in-core one-rank pipeline) and one
      trsm for the rows below it
      A[J0:, J] <- P                               device -> host

Device memory: the panel and two streaming buffers, 3 (n W) words, chosen
to fit the budget; host<->device traffic O(n^3 / W) words, overlapped with
the GEMMs.  288 GB per MI355X makes this the path for n > ~190 000 (fp64).
"""
from __future__ import annotations

import os

import torch

from .. import ops
from ..utils.trace import trace_block
from ._util import conj_trans


def device_budget(dev):
    """Bytes of device memory a factorization may use."""
    v = os.environ.get("SLATE_AMD_DEVICE_BUDGET")
    if v:
        return int(float(v))
    free, _ = torch.cuda.mem_get_info(dev)
    return int(0.85 * free)


def ooc_columns(n, nb, dt, dev):
    """Block-column width W (a multiple of nb) for the out-of-core path, or 0
    when the whole local buffer fits (the in-core path runs)."""
    forced = os.environ.get("SLATE_AMD_OOC_COLS")
    es = torch.empty(0, dtype=dt).element_size()
    if forced:
        return max(nb, int(forced) // nb * nb)
    budget = device_budget(dev)
    if n * n * es <= budget:
        return 0
    W = budget // (3 * n * es) // nb * nb
    return max(nb, W)


def potrf_ooc(H, n, nb, W, dev, la=1):
    """Factor the lower triangle of the host column-major n x n matrix H in
    place (A = L L^H) with block columns of W columns on ``dev``.  Returns
    info (first non-positive pivot column, 1-based) or 0."""
    from ..core.enums import Option, Uplo
    from ..core.matrix import HermitianMatrix
    from ..parallel.comm import self_comm
    from .chol import potrf as _potrf
    dt = H.dtype
    ct = conj_trans(dt)
    cs = torch.cuda.Stream(device=dev)
    cur = torch.cuda.current_stream(dev)
    pinned = H.is_pinned()
    nbuf = [ops.colmajor_empty(n, W, dt, dev) for _ in range(2)]
    panel = ops.colmajor_empty(n, W, dt, dev)
    with trace_block("potrf_ooc"):
        for J0 in range(0, n, W):
            w = min(W, n - J0)
            m = n - J0
            P = panel[:m, :w]
            P.copy_(H[J0:, J0:J0 + w], non_blocking=pinned)
            ev_ready = {}

            def fetch(K0, slot):
                kw = min(W, J0 - K0)
                B = nbuf[slot][:m, :kw]
                with torch.cuda.stream(cs):
                    cs.wait_stream(cur)                 # the buffer's previous GEMM is done
                    B.copy_(H[J0:, K0:K0 + kw], non_blocking=pinned)
                    ev = torch.cuda.Event()
                    ev.record(cs)
                ev_ready[K0] = ev
                return B

            Ks = list(range(0, J0, W))
            bufs = {}
            if Ks:
                bufs[Ks[0]] = fetch(Ks[0], 0)
            for idx, K0 in enumerate(Ks):
                if idx + 1 < len(Ks):
                    bufs[Ks[idx + 1]] = fetch(Ks[idx + 1], (idx + 1) % 2)
                cur.wait_event(ev_ready[K0])
                B = bufs.pop(K0)
                with trace_block("potrf_ooc::update"):
                    # P[0:w] (diagonal block): lower triangle only; rows below: full
                    mask = (1, 1 << 40, 1, 0, 1, 0, 0, 0, 0)
                    ops.gemm(-1.0, B[:w], B[:w], 1.0, P[:w], 'N', ct, mask)
                    if m > w:
                        ops.gemm(-1.0, B[w:], B[:w], 1.0, P[w:], 'N', ct)
            with trace_block("potrf_ooc::panel"):
                D = HermitianMatrix.fromLAPACK(Uplo.Lower, w, P[:w, :w], max(1, panel.stride(1)), nb=nb,
                                               comm=self_comm())
                info = _potrf(D, {Option.Lookahead: la})
                if info:
                    H[J0:, J0:J0 + w].copy_(P)
                    return J0 + info
                if m > w:
                    ops.trsm('R', 'L', ct, 'N', 1.0, P[:w, :w], P[w:])
            H[J0:, J0:J0 + w].copy_(P, non_blocking=pinned)
        cur.synchronize()
    return 0
