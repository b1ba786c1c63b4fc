"""Per-GPU stream/event DAG helpers for lookahead pipelines.

Replaces SLATE's OpenMP task DAG (`#pragma omp task depend(...)` on
per-column sentinels, `src/potrf.cc:84-195`, `src/getrf.cc:81-237`) and its
per-device compute queues (`MatrixStorage.hh:574-609`): a factorization
step is a set of kernels enqueued on

* ``panel``  -- high-priority stream: panel factor, its broadcasts and the
  lookahead-column updates (the critical path),
* ``update`` -- low-priority stream: the bulk trailing update,

with cross-stream dependencies expressed by HIP events recorded after the
producing kernels (no host synchronisation anywhere in a step).  On the CPU
path every call is a no-op and work runs in program order.
"""
from __future__ import annotations

import os
import contextlib

import torch


# the work streams of this process, per device: ONE high-priority panel
# stream, ONE diag stream and ONE update stream, shared by every pipeline
# (potrf, getrf, geqrf, SUMMA, ...) -- with the current stream that is 4
# streams, the box's GPU_MAX_HW_QUEUES default, so no two streams share a
# hardware queue (RCCL kernels of different
# communicators queued behind one another in different orders on different
# ranks can deadlock).
_SHARED = {}
_SHIFT_STREAMS = []        # idle streams of SLATE_AMD_QUEUE_SHIFT (kept alive)
MAX_WORK_STREAMS = 4


class StreamSet:
    _cache = {}

    def __new__(cls, device, n_update=1, reserve_cus=32):
        import os
        reserve_cus = int(os.environ.get("SLATE_AMD_PANEL_CUS", reserve_cus))
        key = (str(device), n_update, reserve_cus, os.environ.get("SLATE_AMD_SERIAL", "0"))
        s = cls._cache.get(key)
        if s is None:
            s = super().__new__(cls)
            s.reserve_cus = reserve_cus
            s._init(torch.device(device), n_update)
            cls._cache[key] = s
        return s

    def _init(self, device, n_update):
        import os
        self.device = device
        self.gpu = device.type == "cuda"
        # SLATE_AMD_SERIAL=1: every pipeline stream IS the current stream (all
        # cross-stream overlap removed) -- the race-detection mode of SURVEY
        # §5.2: a result that changes between serial and pipelined runs
        # points at a missing event dependency.
        self.serial = os.environ.get("SLATE_AMD_SERIAL", "0") == "1"
        if self.gpu and self.serial:
            cur = torch.cuda.current_stream(device)
            self.panel = self.diag = cur
            self.update = [cur] * n_update
        elif self.gpu:
            sh = _SHARED.get(str(device))
            if sh is None:
                # torch: lower number = higher priority; ``diag`` carries the
                # next step's diagonal-tile chain concurrently with the
                # panel's broadcasts (potrf diag-first).
                sh = dict(panel=torch.cuda.Stream(device=device, priority=-1),
                          diag=torch.cuda.Stream(device=device, priority=-1), update={})
                _SHARED[str(device)] = sh
            # ONE update stream per device, shared by every pipeline: with
            # panel, diag and the caller's stream that is 4, the box's
            # hardware queues (one stream per CU reservation made
            # 5, and the high-priority panel stream could share a queue with
            # bulk GEMMs).  A pipeline whose reservation differs from the
            # live stream's replaces it at its fork (_retarget), so the
            # first pipeline's mask never leaks into the next.
            if "upd" not in sh:
                sh["upd"] = (self.reserve_cus, self._update_stream(device, self.reserve_cus))
            self._sh = sh
            self.panel, self.diag = sh["panel"], sh["diag"]
            self.n_update = n_update
        else:
            self.panel = self.diag = None
            self.update = [None] * n_update

    def __getattr__(self, name):
        # ``update`` of a GPU pipeline set: the device's live update stream
        if name == "update" and "_sh" in self.__dict__:
            return [self._sh["upd"][1]] * self.n_update
        raise AttributeError(name)

    # pipelines between a fork and its join, per device (a nested pipeline
    # keeps the live update stream: its outer pipeline still holds it)
    _open = {}

    def _retarget(self):
        """Make the live update stream carry this set's CU reservation.  Only
        outside every open pipeline of the device; the old stream's work is
        drained first (a reservation switch happens once per change of
        factorization kind, never inside a step).  The retired stream is
        PARKED, not destroyed: tensors that outlive their driver (geqrf's T
        factors, ...) may have recorded it with the caching allocator, which
        records an event on it when they are freed.  A parked
        stream carries no work and is reused when its reservation comes
        back, so the process holds at most one stream per reservation and
        drives exactly one update stream."""
        sh = self.__dict__.get("_sh")
        if sh is None or sh["upd"][0] == self.reserve_cus or StreamSet._open.get(str(self.device), 0):
            return
        if torch.cuda.is_current_stream_capturing():
            return                      # capture: keep the live stream (no sync allowed)
        old_res, old = sh["upd"]
        torch.cuda.synchronize(self.device)
        parked = sh.setdefault("parked", {})
        parked[old_res] = old
        new = parked.pop(self.reserve_cus, None)
        if new is None:
            new = self._update_stream(self.device, self.reserve_cus)
        sh["upd"] = (self.reserve_cus, new)

    @staticmethod
    def _update_stream(device, reserve):
        """Bulk-update stream.  By default it is CU-masked to leave
        SLATE_AMD_PANEL_CUS compute units (spread evenly over the 8 XCDs: the
        first mask bits map round-robin to XCDs) free of trailing-update
        workgroups, so the latency-bound panel kernels launched on the
        (unmasked, high-priority) panel stream find idle CUs immediately
        instead of queueing behind long GEMM workgroups (measured on one
        MI355X, n = 32768: dpotrf +12 % with 32 reserved CUs, dgetrf +22 %
        with 64).  SLATE_AMD_PANEL_CUS overrides; 0 disables."""
        if reserve > 0:
            try:
                from .. import _native
                H = _native.hip()
                idx = device.index if device.index is not None else torch.cuda.current_device()
                ncu = H.cu_count(idx)
                if 0 < reserve < ncu:
                    # SLATE_AMD_QUEUE_SHIFT=k (diagnostics): create k idle
                    # streams first, moving the update stream to another of
                    # the box's 4 hardware queues (streams map round-robin)
                    shift = int(os.environ.get("SLATE_AMD_QUEUE_SHIFT", "0"))
                    for _ in range(max(0, shift)):
                        _SHIFT_STREAMS.append(H.stream_create(idx))
                    words = [0] * ((ncu + 31) // 32)
                    for b in range(reserve, ncu):
                        words[b // 32] |= 1 << (b % 32)
                    handle = H.stream_create_cu_mask(idx, words)
                    return torch.cuda.ExternalStream(handle, device=device)
            except Exception as e:  # noqa: BLE001 - plain stream, but say so
                import warnings
                warnings.warn(f"slate_amd: CU-masked update stream unavailable ({e!r}); "
                              "the trailing update shares every CU with the panel kernels", RuntimeWarning)
        return torch.cuda.Stream(device=device, priority=0)

    @classmethod
    def streams_of(cls, device):
        """Every pipeline stream created for ``device`` (distinct objects)."""
        dev = torch.device(device)
        out, seen = [], set()
        for key, ss in cls._cache.items():
            if ss.serial:
                continue          # runs on the caller's stream: not a library stream
            if ss.gpu and ss.device == dev or (ss.gpu and dev.index is None and ss.device.type == dev.type):
                for st in [ss.panel, ss.diag] + list(ss.update):
                    if st is not None and id(st) not in seen:
                        seen.add(id(st))
                        out.append(st)
        return out

    @classmethod
    def census(cls, device):
        """Distinct work streams this process drives on ``device``: the
        pipeline streams plus the current stream."""
        dev = torch.device(device)
        cur = torch.cuda.current_stream(dev) if dev.type == "cuda" else None
        ids = {id(st) for st in cls.streams_of(dev)}
        if cur is not None and not any(st == cur for st in cls.streams_of(dev)):
            ids.add(id(cur))
        return len(ids)

    def check_census(self):
        """Raise if this process drives more work streams on the device than
        the hardware queues it may map them to (MAX_WORK_STREAMS): every
        pipeline stream of the process plus ONE caller stream (whichever
        stream the caller enqueues on).  RCCL adds none: synchronous
        collectives run on the issuing stream (nccl_stream_probe)."""
        if self.gpu and not self.serial:
            cur = torch.cuda.current_stream(self.device)
            n = len([st for st in StreamSet.streams_of(self.device) if st != cur]) + 1
            if n > MAX_WORK_STREAMS:
                from ..core.exceptions import SlateError
                raise SlateError(f"{n} work streams on {self.device} > {MAX_WORK_STREAMS}")
        return self

    def use(self, s):
        if s is None or not self.gpu:
            return contextlib.nullcontext()
        return torch.cuda.stream(s)

    def event(self, s=None):
        """Record an event on stream s (or the current stream)."""
        if not self.gpu:
            return None
        ev = torch.cuda.Event()
        ev.record(s if s is not None else torch.cuda.current_stream(self.device))
        return ev

    def wait(self, s, ev):
        if ev is None or not self.gpu:
            return
        (s if s is not None else torch.cuda.current_stream(self.device)).wait_event(ev)

    def _members(self, diag=True):
        out = []
        for st in [self.panel] + ([self.diag] if diag else []) + list(self.update):
            if all(st is not o for o in out):
                out.append(st)
        return out

    def fork(self, diag=True):
        """All streams wait for the current stream's work so far.  diag=False
        leaves the diag stream out of the fork (and of the matching join): a
        pipeline that never uses it must not open an empty branch, which the
        HIP stream-capture of Option.UseGraph does not survive."""
        if not self.gpu:
            return
        if not self.serial:
            self._retarget()
        self.check_census()
        members = self._members(diag)
        key = str(self.device)
        StreamSet._open[key] = StreamSet._open.get(key, 0) + 1
        if not hasattr(self, "_fstack"):
            self._fstack = []
        self._fstack.append(members)           # fork / join pairs nest
        ev = self.event()
        for st in members:
            st.wait_event(ev)

    def join(self):
        """Current stream waits for all streams."""
        if not self.gpu:
            return
        cur = torch.cuda.current_stream(self.device)
        stack = getattr(self, "_fstack", None)
        if stack:
            key = str(self.device)
            StreamSet._open[key] = max(0, StreamSet._open.get(key, 0) - 1)
        for s in (stack.pop() if stack else self._members()):
            if s != cur:
                cur.wait_event(self.event(s))
