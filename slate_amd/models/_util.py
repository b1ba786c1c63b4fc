"""Shared helpers for the distributed drivers (block-cyclic fast path)."""
from __future__ import annotations

import torch

from ..core.enums import Op, Target, Uplo
from ..core.exceptions import SlateError
from ..core.options import get_option
from ..core.enums import Option
from ..core.storage import DEV, HOST, local_start, l2g
from ..parallel.comm import ProcessGrid


def target_slot(A, opts):
    """Memory slot a driver computes in: Devices -> this rank's GPU."""
    tgt = get_option(opts, Option.Target, None)
    if tgt is None:
        tgt = Target.Devices if A.storage.device.type == "cuda" else Target.HostTask
    if tgt == Target.Devices:
        if not torch.cuda.is_available():
            raise SlateError("Target.Devices requested but no GPU is available")
        return DEV
    return HOST


def grid_of(A) -> ProcessGrid:
    bc = A.storage.bc
    return ProcessGrid(bc.p, bc.q, bc.order, A.storage.comm)


def require_bc(*mats):
    for M in mats:
        if not M.is_block_cyclic() and M.storage.bc is None:
            raise SlateError("this driver requires 2D block-cyclic matrices "
                             "(use slate_amd.redistribute to convert)")


def tiles_local_before(t, p, pr):
    """# of tiles among global tiles [0, t) owned by process row pr."""
    return (t - pr + p - 1) // p if t > pr else 0


def local_rows_from_tile(k, nb, p, pr):
    """Local row index where global tile k (or the first later local tile) starts."""
    return tiles_local_before(k, p, pr) * nb


def uplo_char(u):
    return 'L' if u == Uplo.Lower else ('U' if u == Uplo.Upper else 'G')


def conj_trans(dtype):
    return 'C' if dtype.is_complex else 'T'


def read_to_host(t):
    """Host copy of a (small) device tensor at the END of a driver: a
    non-blocking copy into pinned memory, then one event wait.  This is the
    only point where a factorization waits for the GPU (info values), and it
    is not a torch "synchronizing op" (tests run the drivers under
    torch.cuda.set_sync_debug_mode("error"))."""
    import torch
    if not t.is_cuda:
        return t
    h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    h.copy_(t, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    ev.synchronize()
    return h
