"""Communication layer: one process per MI355X, RCCL over xGMI.

Replaces SLATE's MPI layer (`include/slate/Tile.hh:998-1207`,
`include/slate/BaseMatrix.hh:1762-2452`, `src/internal/internal_comm.cc`).

Design for the 8-GPU xGMI node (every GPU pair has a dedicated link):

* All traffic goes through ``torch.distributed``; with backend ``"nccl"``
  that IS RCCL on ROCm, with device tensors, stream-ordered.  The CPU test
  path uses ``gloo`` with host tensors and the same code.
* Tile broadcasts are issued to *process-row / process-column
  sub-communicators* of the p x q grid (created once per grid and cached),
  never as SLATE's per-tile radix-2/4 hypercube trees of point-to-point
  messages: on a fully connected xGMI mesh a collective over the row or
  column group moves each byte over one hop and RCCL pipelines it over the
  links.  Panels are packed into ONE contiguous buffer per step so each
  step is one collective (few, large messages -- xGMI links are ~150 GB/s
  each, latency ~10 us per collective).
* Small reductions (norms, info, pivot MAXLOC) are packed into one tensor
  per call.  MAXLOC has no RCCL op: it is an all-gather of (value, index)
  pairs followed by a local arg-max (deterministic tie-break on the lowest
  index, NaN wins -- same as SLATE's `mpi_max_nan`).
* ``Comm`` with size 1 short-circuits every call (no process group needed),
  so the single-GPU bench path has zero communication overhead.

Issue order across communicators (why the pipelines cannot deadlock)
--------------------------------------------------------------------
A pipelined driver issues collectives on several communicators from
several HIP streams: e.g. distributed potrf uses ``col_comm`` on the panel
stream, ``row_comm`` on the diag stream and ``col_comm_u`` (same members as
``col_comm``, its own RCCL communicator) on the update stream.  torch runs a
synchronous RCCL collective on the issuing stream, and with
GPU_MAX_HW_QUEUES=4 two of those streams may share one hardware queue, whose
packets execute in submission order.  So two ranks that submitted two
collectives of different communicators in OPPOSITE orders into one shared
queue would each wait inside the first for the other: a deadlock no timeout
on a single communicator explains.

The drivers rule that out by construction: every rank runs the same
deterministic step loop, and the collectives of step t are issued in one
fixed global sequence (potrf: column broadcast of the diagonal tile, the row
broadcast chunks, the panel-stream column gathers, then the update-stream
column gathers) of which each rank issues the subsequence it is a member
of -- rank-dependent branches (``own_col``, ``own_diag``) only select
compute, or select whole collectives for ALL members of their communicator
alike (``own_col`` is the same on every member of ``col_comm``).  Hence all
ranks' issue orders are restrictions of one total order, so whatever
queue sharing HIP picks, the earliest unfinished collective in that order has
nothing unfinished ahead of it in any member's queue except compute (which
finishes) -- it completes, and induction covers the rest.  Cross-stream
event waits only point backwards in issue order, so they keep the argument.
``ORDER_LOG`` records, per rank, the (communicator, sequence number) of
every collective in issue order; tests/test_comm_order.py gathers the logs of
gloo 2x2 / 2x4 runs of potrf, getrf, geqrf and gemm and checks that their
union is acyclic (one global order exists).  All sub-communicators of a grid,
the update stream's included, are created eagerly in ``ProcessGrid``: RCCL
communicator creation is itself collective over the world and must not run
interleaved with a pipeline's in-flight collectives.
"""
from __future__ import annotations

import os
from typing import Optional, Sequence

import torch
import torch.distributed as dist

from ..core.exceptions import CommError
from ..utils import watchdog as _wd


# per-communicator issuing streams while "on" (tests: one stream per comm)
STREAM_LOG = {"on": False, "used": {}}
# issue-order log while "on": ((members, tag), kind, seq) per collective or
# matched point-to-point pair, in this rank's issue order (tests)
ORDER_LOG = {"on": False, "ops": [], "seq": {}}


def _order(key, kind):
    if ORDER_LOG["on"]:
        n = ORDER_LOG["seq"].get(key, 0)
        ORDER_LOG["seq"][key] = n + 1
        ORDER_LOG["ops"].append((key, kind, n))


def _dist_ready() -> bool:
    return dist.is_available() and dist.is_initialized()


class Comm:
    """A communicator: the world or a sub-group of ranks.

    ``ranks`` are world ranks in communicator order; ``rank`` is this
    process's index inside the communicator (or -1 if not a member).
    """

    def __init__(self, group=None, ranks: Optional[Sequence[int]] = None):
        if _dist_ready():
            world = dist.get_world_size()
            self.world_rank = dist.get_rank()
            if ranks is None:
                ranks = list(range(world))
            self.ranks = list(ranks)
            self.group = group
        else:
            self.world_rank = 0
            self.ranks = [0] if ranks is None else list(ranks)
            self.group = None
        self.size = len(self.ranks)
        self.rank = self.ranks.index(self.world_rank) if self.world_rank in self.ranks else -1
        self.backend = dist.get_backend(self.group) if (_dist_ready() and self.size > 1) else "self"
        self._subcache = {}
        self.tag = ""

    # -- helpers ---------------------------------------------------------
    def _g(self, r):
        return self.ranks[r]

    def _key(self):
        return (tuple(self.ranks), getattr(self, "tag", ""))

    def _ord(self, kind, peer=None):
        """Issue-order log (module docstring): collectives are keyed by the
        communicator, point-to-point traffic by the communicator and the
        (unordered) rank pair."""
        if ORDER_LOG["on"] and self.size > 1:
            if peer is None:
                _order(self._key(), kind)
            else:
                a, b = sorted((self.world_rank, self._g(peer)))
                _order(self._key() + (a, b), "p2p")

    def _note(self, t):
        """Stream log (tests): torch runs a synchronous RCCL collective on
        the ISSUING stream (profiles/r4/nccl_stream_probe.txt), so the
        drivers keep each communicator on one stream -- its collectives
        then keep one order on every rank and add no hardware queue.  While
        STREAM_LOG is enabled, record which streams issued on this comm."""
        if STREAM_LOG["on"] and isinstance(t, torch.Tensor) and t.is_cuda and self.size > 1:
            STREAM_LOG["used"].setdefault(id(self), set()).add(torch.cuda.current_stream(t.device).cuda_stream)

    def _prep(self, t: torch.Tensor):
        """gloo cannot move device tensors and RCCL cannot move host ones."""
        if self.backend == "gloo" and t.is_cuda:
            return t.cpu(), True
        if self.backend == "nccl" and not t.is_cuda:
            return t.cuda(), True
        return t, False

    @staticmethod
    def _flat_view(t: torch.Tensor):
        """A contiguous alias of t's memory when one exists (column-major
        matrices with ld == rows are contiguous as their transpose), else None."""
        if t.is_contiguous():
            return t
        if t.dim() == 2 and t.stride(0) == 1 and (t.stride(1) == t.shape[0] or t.shape[1] <= 1):
            v = t.t()
            if v.is_contiguous():
                return v
        return None

    def _finish(self, t, staged, orig):
        if staged:
            orig.copy_(t)

    def __repr__(self):
        return f"Comm(size={self.size}, rank={self.rank}, backend={self.backend})"

    # -- collectives -----------------------------------------------------
    @_wd.watched("comm.barrier")
    def barrier(self):
        _wd.beat("comm.barrier")
        self._ord("barrier")
        if self.size > 1:
            if self.backend == "nccl":
                # device-side barrier: tiny allreduce on the current stream
                t = torch.zeros(1, device="cuda")
                dist.all_reduce(t, group=self.group)
            else:
                dist.barrier(group=self.group)

    @_wd.watched("comm.bcast")
    def bcast(self, t: torch.Tensor, root: int, async_op=False):
        """Broadcast t from comm-rank root (in place)."""
        _wd.beat("comm.bcast")
        self._note(t)
        self._ord("bcast")
        if self.size == 1:
            return None
        try:
            fv = self._flat_view(t)
            src = fv if fv is not None else t.contiguous()
            x, staged = self._prep(src)
            w = dist.broadcast(x, src=self._g(root), group=self.group, async_op=async_op)
            if async_op and not staged and x is src and fv is not None:
                return w
            if async_op:
                w.wait()
            if x is not src:          # staged through host/device
                src.copy_(x)
            if fv is None:            # broadcast into a contiguous copy
                t.copy_(src)
            return None
        except Exception as e:  # noqa: BLE001
            raise CommError(f"bcast failed: {e}") from e

    @_wd.watched("comm.bcast_sa")
    def bcast_sa(self, t: torch.Tensor, root: int):
        """Broadcast t from comm-rank root in two DIRECT phases -- scatter
        (the root sends piece j of t to member j) then all-gather (every
        member sends its piece to every other member) -- as grouped
        point-to-point transfers.  On the xGMI mesh every GPU pair has its
        own link, so each link carries 2 B / size bytes instead of the B of
        a ring / tree broadcast and a receiver ingests over size - 1 links at
        once (profiles/r6/critpath_2x4_links.md).  size <= 2: plain bcast.
        One issue-order key, like bcast (the two phases are issued by every
        member in the same order)."""
        _wd.beat("comm.bcast_sa")
        self._note(t)
        if self.size <= 2:
            return self.bcast(t, root)
        self._ord("bcast")
        try:
            fv = self._flat_view(t)
            src = fv if fv is not None else t.contiguous()
            x, staged = self._prep(src)
            flat = x.reshape(-1)
            n, P, me = flat.numel(), self.size, self.rank
            L = -(-n // P)

            def piece(j):
                return flat[min(n, j * L):min(n, (j + 1) * L)]

            def run(ops):
                if ops:
                    for w in dist.batch_isend_irecv(ops):
                        w.wait()
            # phase 1: scatter from the root
            ops = []
            if me == root:
                ops = [dist.P2POp(dist.isend, piece(j), self._g(j), self.group)
                       for j in range(P) if j != root and piece(j).numel()]
            elif piece(me).numel():
                ops = [dist.P2POp(dist.irecv, piece(me), self._g(root), self.group)]
            run(ops)
            # phase 2: every rank's piece to every member except itself and
            # the root (which holds everything); the root sends its own piece
            ops = []
            for k in range(P):
                if k == me or k == root:
                    continue
                if piece(me).numel():
                    ops.append(dist.P2POp(dist.isend, piece(me), self._g(k), self.group))
            if me != root:
                for r in range(P):
                    if r != me and piece(r).numel():
                        ops.append(dist.P2POp(dist.irecv, piece(r), self._g(r), self.group))
            run(ops)
            if x is not src:
                src.copy_(x)
            if fv is None:
                t.copy_(src)
            return None
        except Exception as e:  # noqa: BLE001
            raise CommError(f"bcast_sa failed: {e}") from e

    @_wd.watched("comm.allreduce")
    def allreduce(self, t: torch.Tensor, op: str = "sum"):
        _wd.beat("comm.allreduce")
        self._note(t)
        self._ord("allreduce")
        if self.size == 1:
            return t
        rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX,
               "min": dist.ReduceOp.MIN, "prod": dist.ReduceOp.PRODUCT}[op]
        fv = self._flat_view(t)
        src = fv if fv is not None else t.contiguous()
        x, staged = self._prep(src)
        if op == "max" and x.dtype.is_floating_point:
            # NaN-propagating max (SLATE mpi_max_nan): reduce a NaN flag too.
            nanflag = torch.isnan(x).to(x.dtype)
            dist.all_reduce(nanflag, op=dist.ReduceOp.MAX, group=self.group)
            dist.all_reduce(x, op=rop, group=self.group)
            x.copy_(torch.where(nanflag > 0, torch.full_like(x, float("nan")), x))
        else:
            dist.all_reduce(x, op=rop, group=self.group)
        if x is not src:              # staged through host/device
            src.copy_(x)
        if fv is None:                # reduced a contiguous copy
            t.copy_(src)
        return t

    @_wd.watched("comm.allreduce_scalar")
    def allreduce_scalar(self, v, op="sum", dtype=torch.float64, device=None):
        if self.size == 1:
            return v
        dev = device or ("cuda" if self.backend == "nccl" else "cpu")
        t = torch.tensor([v], dtype=dtype, device=dev)
        self.allreduce(t, op)
        return t.item()

    @_wd.watched("comm.maxloc")
    def maxloc(self, value: float, index: int):
        """Global (max value, index of max) over ranks; NaN wins, ties -> lowest index."""
        if self.size == 1:
            return value, index
        self._ord("maxloc")
        dev = "cuda" if self.backend == "nccl" else "cpu"
        t = torch.tensor([[float(value), float(index)]], dtype=torch.float64, device=dev)
        out = [torch.empty_like(t) for _ in range(self.size)]
        dist.all_gather(out, t, group=self.group)
        best_v, best_i = None, None
        for o in out:
            v, i = o[0, 0].item(), int(o[0, 1].item())
            if best_v is None or (v != v and best_v == best_v) or v > best_v or (v == best_v and i < best_i):
                best_v, best_i = v, i
        return best_v, best_i

    @_wd.watched("comm.allgather")
    def allgather(self, t: torch.Tensor) -> torch.Tensor:
        """Concatenate equal-size tensors from all ranks along a new dim 0."""
        _wd.beat("comm.allgather")
        self._note(t)
        self._ord("allgather")
        if self.size == 1:
            return t.unsqueeze(0)
        x, _ = self._prep(t.contiguous())
        if x.numel() == 0:
            return torch.empty((self.size,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        x = x.reshape((-1,) + tuple(x.shape[1:])) if x.dim() else x.reshape(1)
        flat = torch.empty((self.size * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        if self.backend == "gloo":
            dist.all_gather(list(flat.chunk(self.size)), x, group=self.group)
        else:
            dist.all_gather_into_tensor(flat, x, group=self.group)
        out = flat.view((self.size,) + tuple(t.shape))
        return out.to(t.device) if out.device != t.device else out

    @_wd.watched("comm.allgatherv")
    def allgatherv(self, t: torch.Tensor) -> list:
        """All-gather of variable-length 1-D tensors (SLATE stedc Allgatherv)."""
        _wd.beat("comm.allgatherv")
        self._note(t)
        if self.size == 1:
            return [t]
        x, _ = self._prep(t.contiguous().reshape(-1))
        n = torch.tensor([x.numel()], dtype=torch.int64, device=x.device)
        ns = self.allgather(n).reshape(-1).tolist()
        mx = max(ns)
        buf = torch.zeros(mx, dtype=x.dtype, device=x.device)
        buf[: x.numel()] = x
        allb = self.allgather(buf)
        return [allb[r, : ns[r]].to(t.device) for r in range(self.size)]

    @_wd.watched("comm.reduce")
    def reduce(self, t: torch.Tensor, root: int, op="sum"):
        _wd.beat("comm.reduce")
        self._note(t)
        self._ord("reduce")
        if self.size == 1:
            return t
        x, staged = self._prep(t.contiguous())
        dist.reduce(x, dst=self._g(root), op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX,
                    group=self.group)
        if x is not t and self.rank == root:
            t.copy_(x)
        return t

    @_wd.watched("comm.send")
    def send(self, t: torch.Tensor, dst: int, tag: int = 0):
        _wd.beat("comm.send")
        self._note(t)
        self._ord("p2p", dst)
        if self.size == 1:
            return
        x, _ = self._prep(t.contiguous())
        dist.send(x, dst=self._g(dst), group=self.group, tag=tag) if self.backend != "nccl" else \
            dist.send(x, dst=self._g(dst), group=self.group)

    @_wd.watched("comm.recv")
    def recv(self, t: torch.Tensor, src: int, tag: int = 0):
        _wd.beat("comm.recv")
        self._note(t)
        self._ord("p2p", src)
        if self.size == 1:
            return t
        x, _ = self._prep(t if t.is_contiguous() else t.contiguous())
        if self.backend != "nccl":
            dist.recv(x, src=self._g(src), group=self.group, tag=tag)
        else:
            dist.recv(x, src=self._g(src), group=self.group)
        if x is not t:
            t.copy_(x)
        return t

    @_wd.watched("comm.sendrecv")
    def sendrecv(self, send_t: torch.Tensor, dst: int, recv_t: torch.Tensor, src: int):
        """Simultaneous exchange (MPI_Sendrecv) via batched p2p."""
        _wd.beat("comm.sendrecv")
        self._note(send_t)
        for r in sorted({dst, src}):
            self._ord("p2p", r)
        if self.size == 1:
            recv_t.copy_(send_t)
            return recv_t
        xs, _ = self._prep(send_t.contiguous())
        xr, _ = self._prep(torch.empty_like(recv_t).contiguous())
        ops = [dist.P2POp(dist.isend, xs, self._g(dst), self.group),
               dist.P2POp(dist.irecv, xr, self._g(src), self.group)]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        recv_t.copy_(xr)
        return recv_t

    @_wd.watched("comm.exchange")
    def exchange(self, sends: dict, recvs: dict):
        """Batched point-to-point: sends {dst: tensor}, recvs {src: tensor}."""
        _wd.beat("comm.exchange")
        for t in list(sends.values()) + list(recvs.values()):
            self._note(t)
        for r in sorted(set(sends) | set(recvs)):
            self._ord("p2p", r)
        if self.size == 1 or (not sends and not recvs):
            return
        ops, fix = [], []
        for d, t in sends.items():
            x, _ = self._prep(t.contiguous())
            ops.append(dist.P2POp(dist.isend, x, self._g(d), self.group))
        for s, t in recvs.items():
            x, staged = self._prep(t if t.is_contiguous() else t.contiguous())
            ops.append(dist.P2POp(dist.irecv, x, self._g(s), self.group))
            if x is not t:
                fix.append((x, t))
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        for x, t in fix:
            t.copy_(x)

    @_wd.watched("comm.bcast_object")
    def bcast_object(self, obj, root: int):
        if self.size == 1:
            return obj
        self._ord("bcast_object")
        lst = [obj]
        dist.broadcast_object_list(lst, src=self._g(root), group=self.group)
        return lst[0]

    # -- sub-communicators -----------------------------------------------
    def split(self, color_of_rank: Sequence[int], tag: str = ""):
        """Collectively create sub-communicators: ranks with equal color share
        one.  Every member must call with the same list (MPI_Comm_split).
        A different ``tag`` creates a second, independent communicator over
        the same members (RCCL serialises the collectives of one communicator
        on one internal stream: a pipeline's panel stream and update stream
        each get their own, so a panel broadcast never queues behind a
        trailing-update exchange)."""
        key = (tuple(color_of_rank), tag)
        if key in self._subcache:
            return self._subcache[key]
        colors = sorted(set(color_of_rank))
        mine = None
        for c in colors:
            members = [self.ranks[r] for r in range(self.size) if color_of_rank[r] == c]
            if self.size > 1 and len(members) > 1:
                g = dist.new_group(members, backend=None)
            else:
                g = None
            if self.rank >= 0 and color_of_rank[self.rank] == c:
                mine = Comm(g, members) if len(members) > 1 else _SelfComm(self.world_rank)
                mine.tag = tag
        self._subcache[key] = mine
        return mine


class _SelfComm(Comm):
    def __init__(self, world_rank=0):
        self.world_rank = world_rank
        self.ranks = [world_rank]
        self.group = None
        self.size = 1
        self.rank = 0
        self.backend = "self"
        self._subcache = {}


class LoopbackComm(Comm):
    """Rehearsal transport: ONE process plays world rank ``rank`` of a
    ``size``-rank job (SLATE_AMD_LOOPBACK=size:rank, or ``loopback()``).
    Every collective becomes a same-size local device copy on the issuing
    stream -- the bytes a real collective would land in this rank's buffers
    -- so the rank's own kernel DAG runs at its true local shapes and
    stream order on one GPU; received data is this rank's own (values, not
    the peers').  ``LOG`` records (op, communicator size, bytes, stream
    handle) for the communication-cost model of tools/r5/loopback_critpath.py."""

    LOG: list = []
    _scratch: dict = {}

    def __init__(self, size, rank, ranks=None):
        self.world_rank = rank
        self.ranks = list(range(size)) if ranks is None else list(ranks)
        self.size = len(self.ranks)
        self.rank = self.ranks.index(rank) if rank in self.ranks else -1
        self.group = None
        self.backend = "loopback"
        self._subcache = {}

    # SLATE_AMD_LOOPBACK_LINK="alpha_us,beta_GBps": every collective also
    # holds its issuing stream for its modelled duration (a one-wave spin
    # kernel, ops.spin_ns) -- the link cost then lands where the DAG puts
    # it: overlapped behind other streams' kernels or on the critical chain,
    # instead of being added up afterwards.  bcast / reduce: alpha + B/beta;
    # allreduce: alpha + 2 B/beta; allgather(v): alpha + (P-1) B/beta.
    _link = None
    # bytes on the BUSIEST link per byte of the message (ring / pipelined
    # tree collectives: every link of the ring carries the whole message;
    # bcast_sa: 2 / size, see Comm.bcast_sa); bcast_sa pays alpha twice
    _LINK_FACTOR = {"bcast": 1.0, "reduce": 1.0, "allreduce": 2.0}

    @classmethod
    def link(cls):
        if cls._link is None:
            e = os.environ.get("SLATE_AMD_LOOPBACK_LINK", "")
            cls._link = (False,)
            if e:
                a, b = (float(x) for x in e.split(",")[:2])
                cls._link = (True, a * 1e-6, b * 1e9)
        return cls._link

    def _log(self, op, t):
        nbytes = t.numel() * t.element_size() if isinstance(t, torch.Tensor) else 0
        st = torch.cuda.current_stream(t.device).cuda_stream if isinstance(t, torch.Tensor) and t.is_cuda else 0
        LoopbackComm.LOG.append((op, self.size, nbytes, st))
        lk = self.link()
        if lk[0] and isinstance(t, torch.Tensor) and t.is_cuda and self.size > 1:
            if op == "bcast_sa":
                f, a = 2.0 / self.size, 2 * lk[1]
            else:
                f, a = self._LINK_FACTOR.get(op, float(self.size - 1)), lk[1]
            from .. import ops
            ops.spin_ns((a + f * nbytes / lk[2]) * 1e9, t)

    @classmethod
    def _tmp(cls, t):
        key = (str(t.device), t.dtype)
        buf = cls._scratch.get(key)
        if buf is None or buf.numel() < t.numel():
            buf = cls._scratch[key] = torch.empty(max(t.numel(), 1 << 16), dtype=t.dtype, device=t.device)
        return buf[: t.numel()]

    def _land(self, t):
        """t receives its own bytes again: one read + one write of t (not
        with the link model, whose spin stands for the whole transfer)."""
        if t.numel() == 0 or self.link()[0]:
            return t
        fv = self._flat_view(t)
        src = fv.reshape(-1) if fv is not None else t.contiguous().reshape(-1)
        tmp = self._tmp(src)
        tmp.copy_(src)
        if fv is not None:
            src.copy_(tmp)
        else:
            t.copy_(tmp.view(t.shape))
        return t

    def barrier(self):
        return None

    def bcast(self, t, root, async_op=False):
        self._log("bcast", t)
        if self.size > 1 and self.rank != root:
            self._land(t)
        return None

    def bcast_sa(self, t, root):
        if self.size <= 2:
            return self.bcast(t, root)
        self._log("bcast_sa", t)
        if self.rank != root:
            self._land(t)
        return None

    def allreduce(self, t, op="sum"):
        self._log("allreduce", t)
        if self.size > 1:
            self._land(t)
        return t

    def allreduce_scalar(self, v, op="sum", dtype=torch.float64, device=None):
        return v

    def maxloc(self, value, index):
        return value, index

    def allgather(self, t):
        self._log("allgather", t)
        return t.unsqueeze(0).expand((self.size,) + tuple(t.shape)).contiguous()

    def allgatherv(self, t):
        self._log("allgatherv", t)
        return [t.clone() for _ in range(self.size)]

    def reduce(self, t, root, op="sum"):
        self._log("reduce", t)
        if self.size > 1 and self.rank == root:
            self._land(t)
        return t

    def send(self, t, dst, tag=0):
        self._log("send", t)

    def recv(self, t, src, tag=0):
        self._log("recv", t)
        return self._land(t) if self.size > 1 else t

    def sendrecv(self, send_t, dst, recv_t, src):
        self._log("sendrecv", recv_t)
        if recv_t.shape == send_t.shape:
            recv_t.copy_(send_t)
        else:
            self._land(recv_t)
        return recv_t

    def exchange(self, sends, recvs):
        pool = {}
        for t in sends.values():
            pool.setdefault(t.numel(), t)
        for t in recvs.values():
            self._log("exchange", t)
            d = pool.get(t.numel())
            if d is not None and d.dtype == t.dtype:
                t.copy_(d.reshape(t.shape) if d.is_contiguous() else d.contiguous().reshape(t.shape))
            else:
                self._land(t)

    def bcast_object(self, obj, root):
        return obj

    def split(self, color_of_rank, tag=""):
        key = (tuple(color_of_rank), tag)
        if key in self._subcache:
            return self._subcache[key]
        mine = None
        if self.rank >= 0:
            c = color_of_rank[self.rank]
            members = [self.ranks[r] for r in range(self.size) if color_of_rank[r] == c]
            mine = LoopbackComm(0, self.world_rank, members) if len(members) > 1 else _SelfComm(self.world_rank)
        self._subcache[key] = mine
        return mine


_WORLD = None


def loopback(size: int, rank: int) -> Comm:
    """Make the world a LoopbackComm (this process plays ``rank`` of ``size``)."""
    global _WORLD
    _WORLD = LoopbackComm(size, rank)
    ProcessGrid._cache.clear()
    return _WORLD


def self_comm() -> Comm:
    """This rank alone (rank-local matrices inside multi-rank drivers)."""
    me = dist.get_rank() if _dist_ready() else 0
    return _SelfComm(me)


def world() -> Comm:
    """The global communicator (all ranks; a size-1 comm without torch.distributed)."""
    global _WORLD
    if isinstance(_WORLD, LoopbackComm):
        return _WORLD
    lb = os.environ.get("SLATE_AMD_LOOPBACK")
    if lb and _WORLD is None:
        size, rank = (int(x) for x in lb.split(":"))
        _WORLD = LoopbackComm(size, rank)
        return _WORLD
    if _WORLD is None or (_dist_ready() and _WORLD.size != dist.get_world_size()):
        _WORLD = Comm() if _dist_ready() else _SelfComm(0)
    return _WORLD


def init(backend: Optional[str] = None):
    """Initialise torch.distributed from the torchrun environment (RANK,
    WORLD_SIZE, MASTER_ADDR/PORT, LOCAL_RANK) and bind this process to its
    GPU.  Backend defaults to "nccl" (= RCCL) when GPUs are present;
    SLATE_AMD_DIST_BACKEND=gloo forces gloo (rehearsing several ranks on one
    GPU: every rank then uses the current device)."""
    if not _dist_ready() and int(os.environ.get("WORLD_SIZE", "1")) > 1:
        if backend is None:
            backend = os.environ.get("SLATE_AMD_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        # explicit collective timeout: RCCL's watchdog aborts a collective
        # stuck past it (a dead or deadlocked peer) instead of hanging the job
        from datetime import timedelta
        tmo = timedelta(seconds=float(os.environ.get("SLATE_AMD_COMM_TIMEOUT", "600")))
        if backend == "nccl":
            lr = int(os.environ.get("LOCAL_RANK", "0"))
            torch.cuda.set_device(lr)
            dist.init_process_group(backend, device_id=torch.device("cuda", lr), timeout=tmo)
        else:
            dist.init_process_group(backend, timeout=tmo)
    elif torch.cuda.is_available() and "LOCAL_RANK" in os.environ:
        torch.cuda.set_device(int(os.environ["LOCAL_RANK"]))
    global _WORLD
    _WORLD = None
    _wd.from_env()
    return world()


def finalize():
    global _WORLD
    from .peer import PeerMailbox
    if PeerMailbox._live:
        if _dist_ready():
            dist.barrier()            # every peer's kernels are done with my mailbox
        PeerMailbox.release_all()
    if _dist_ready():
        dist.destroy_process_group()
    _WORLD = None


class ProcessGrid:
    """p x q grid over a communicator with row/column sub-communicators.

    Rank mapping follows `func.process_2d_grid(order, p, q)`: Col order =>
    rank = pr + pc*p.  ``row_comm`` spans the ranks of this process row
    (indexed by pc), ``col_comm`` those of this process column (indexed by pr).
    """

    _cache = {}

    def __new__(cls, p, q, order="C", comm: Optional[Comm] = None):
        comm = comm or world()
        key = (p, q, str(order), tuple(comm.ranks))
        g = cls._cache.get(key)
        if g is not None:
            return g
        g = super().__new__(cls)
        g._init(p, q, str(order), comm)
        cls._cache[key] = g
        return g

    def _init(self, p, q, order, comm):
        from ..core.enums import GridOrder
        if p * q != comm.size:
            raise CommError(f"grid {p}x{q} does not match communicator size {comm.size}")
        self.p, self.q, self.comm = p, q, comm
        self.order = GridOrder.from_string(order)
        r = comm.rank
        self.pr, self.pc = self.coords(r)
        rows = [self.coords(x)[0] for x in range(comm.size)]
        cols = [self.coords(x)[1] for x in range(comm.size)]
        # row_comm: same process row (members ordered by pc)
        self.row_comm = comm.split(rows)
        self.col_comm = comm.split(cols)
        self._rows, self._cols = rows, cols
        # the update stream's column communicator, created HERE with the
        # others (not lazily inside a pipeline: communicator creation is a
        # world collective, see the module docstring)
        self._col_comm_u = comm.split(cols, tag="update") if p > 1 else self.col_comm

    @property
    def col_comm_u(self):
        """Second column communicator, for collectives issued from the
        low-priority update stream."""
        return self._col_comm_u

    def coords(self, rank):
        from ..core.enums import GridOrder
        if self.order == GridOrder.Col:
            return rank % self.p, rank // self.p
        return rank // self.q, rank % self.q

    def rank_of(self, pr, pc):
        from ..core.enums import GridOrder
        if self.order == GridOrder.Col:
            return pr + pc * self.p
        return pr * self.q + pc

    def __repr__(self):
        return f"ProcessGrid({self.p}x{self.q}, order={self.order}, pr={self.pr}, pc={self.pc})"
