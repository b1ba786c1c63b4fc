"""Peer-mapped device mailboxes: in-kernel communication between the GPUs of
one communicator without the host.

Each rank allocates a small uncached device buffer (hipExtMallocWithFlags
with hipDeviceMallocUncached: every access reaches memory, which an
in-kernel cross-device hand-off needs), exports it with hipIpcGetMemHandle,
and opens every peer's buffer with hipIpcOpenMemHandle -- over xGMI on an
8-GPU node, the same HBM when ranks share one GPU (the rehearsals of
tests/test_dist_gpu.py).  The 64-byte handles travel once, over the
communicator itself.  A kernel then stores straight into the peers'
mailboxes (system-scope stores, a release fence, then a sequence tag) and
polls its own (device-side exchange for tiny messages;
SLATE issues MPI_Allreduce/MPI_Bcast per pivot column from host threads,
src/internal/Tile_getrf.hh:267-320).

Used by the distributed LU panel (models/lu.py `_panel_pp_dist`,
csrc/hip/lu_dist.hip `lu_dist_base_kernel`): one persistent launch per
b-column block replaces b host-issued kernels + b record all-gathers.
"""
from __future__ import annotations

import os

import torch


class PeerMailbox:
    """Mailboxes of one communicator on one device (created collectively,
    cached per communicator)."""

    _live: list = []

    @classmethod
    def of(cls, comm, device):
        """The communicator's mailbox on ``device`` (kept on the communicator
        object, so a new communicator never inherits a stale one)."""
        if comm.__dict__.get("_peer_mailbox_dead"):
            from ..core.exceptions import SlateError
            raise SlateError("peer mailboxes of this communicator timed out earlier; their sequence tags no longer "
                             "agree across ranks -- build a new process grid (communicator) to continue")
        boxes = comm.__dict__.setdefault("_peer_mailboxes", {})
        mb = boxes.get(str(device))
        if mb is None:
            mb = boxes[str(device)] = cls(comm, device)
            cls._live.append(mb)
        return mb

    @staticmethod
    def enabled(comm, t: torch.Tensor) -> bool:
        """Device mailboxes for this communicator and tensor: GPU tensors,
        2 <= size <= the kernel's peer limit; SLATE_AMD_LU_PEER=0 keeps the
        host-issued record all-gather."""
        if os.environ.get("SLATE_AMD_LU_PEER", "1") == "0" or not t.is_cuda or comm.size < 2 or \
                getattr(comm, "backend", "") == "loopback":
            return False
        from .. import _native
        return comm.size <= _native.hip().lu_peer_sizes()[3]

    def __init__(self, comm, device):
        from .. import _native
        H = _native.hip()
        self.H = H
        self.comm = comm
        self.device = torch.device(device)
        mb_bytes, part_bytes, self.bmax, self.pmax = H.lu_peer_sizes()
        with torch.cuda.device(self.device):
            self.own, handle = H.lu_peer_alloc(mb_bytes)
        h = torch.frombuffer(bytearray(handle), dtype=torch.uint8).clone()
        if comm.backend == "nccl":
            h = h.to(self.device)
        allh = comm.allgather(h).cpu()                       # (p, 64)
        self.opened = []
        ptrs = []
        for r in range(comm.size):
            if r == comm.rank:
                ptrs.append(self.own)
            else:
                ptr = H.lu_peer_open(bytes(allh[r].tolist()))
                self.opened.append(ptr)
                ptrs.append(ptr)
        self.mbox = torch.tensor(ptrs, dtype=torch.int64, device=self.device)
        self.part = torch.zeros(part_bytes, dtype=torch.uint8, device=self.device)
        self.err = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.seq = 0
        self.launches = 0
        torch.cuda.synchronize(self.device)
        comm.barrier()                                       # every peer's mailbox is mapped

    def next_seq(self, ncols: int) -> int:
        """Sequence base of the next base block of ncols columns (every rank
        of the communicator issues the same sequence of blocks)."""
        s = self.seq
        self.seq += ncols + 1
        self.launches += 1
        return s

    def check(self):
        """Raise if a kernel of this communicator timed out waiting for a peer
        (reads one device word: call where the driver synchronises anyway).
        The error word is sticky and the ranks' host sequence counters may no
        longer agree after a timeout, so the communicator is marked: every
        later use of its mailboxes raises instead of waiting on tags that
        never come.  The mapped buffers stay allocated -- a peer
        may still store into them -- until release_all() at finalize."""
        if int(self.err.item()) != 0:
            from ..core.exceptions import SlateError
            self.comm.__dict__["_peer_mailbox_dead"] = True
            self.comm.__dict__.pop("_peer_mailboxes", None)
            raise SlateError("peer mailbox exchange timed out (a column peer never posted its record); "
                             "this communicator's mailboxes are retired")

    def close(self):
        torch.cuda.synchronize(self.device)
        for ptr in self.opened:
            self.H.lu_peer_close(ptr)
        self.opened = []
        if self.own:
            self.H.lu_peer_free(self.own)
            self.own = 0

    @classmethod
    def release_all(cls):
        """Unmap and free every mailbox of the process (after the device work
        of this rank; a peer's mapping keeps its pages until it closes it)."""
        for mb in cls._live:
            try:
                mb.close()
            except Exception:  # noqa: BLE001 - best effort at teardown
                pass
            mb.comm.__dict__.pop("_peer_mailboxes", None)
        cls._live.clear()
