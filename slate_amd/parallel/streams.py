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

import contextlib

import torch


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
            # torch: lower number = higher priority; ``diag`` carries the
            # next step's diagonal-tile chain concurrently with the panel's
            # broadcasts (potrf diag-first)
            self.panel = torch.cuda.Stream(device=device, priority=-1)
            self.diag = torch.cuda.Stream(device=device, priority=-1)
            self.update = [self._update_stream(device, self.reserve_cus) for _ in range(n_update)]
        else:
            self.panel = self.diag = None
            self.update = [None] * n_update

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
            if ss.gpu and ss.device == dev or (ss.gpu and dev.index is None and ss.device.type == dev.type):
                for st in [ss.panel, ss.diag] + list(ss.update):
                    if st is not None and id(st) not in seen:
                        seen.add(id(st))
                        out.append(st)
        return out

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

    def fork(self):
        """All streams wait for the current stream's work so far."""
        if not self.gpu:
            return
        ev = self.event()
        self.panel.wait_event(ev)
        if self.diag is not self.panel:
            self.diag.wait_event(ev)
        for u in self.update:
            u.wait_event(ev)

    def join(self):
        """Current stream waits for all streams."""
        if not self.gpu:
            return
        cur = torch.cuda.current_stream(self.device)
        for s in [self.panel, self.diag] + self.update:
            cur.wait_event(self.event(s))
