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

    def __new__(cls, device, n_update=1):
        key = (str(device), n_update)
        s = cls._cache.get(key)
        if s is None:
            s = super().__new__(cls)
            s._init(torch.device(device), n_update)
            cls._cache[key] = s
        return s

    def _init(self, device, n_update):
        self.device = device
        self.gpu = device.type == "cuda"
        if self.gpu:
            hi, lo = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (-1, 0)
            # torch: lower number = higher priority
            self.panel = torch.cuda.Stream(device=device, priority=-1)
            self.update = [torch.cuda.Stream(device=device, priority=0) for _ in range(n_update)]
        else:
            self.panel = None
            self.update = [None] * n_update

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
        for u in self.update:
            u.wait_event(ev)

    def join(self):
        """Current stream waits for all streams."""
        if not self.gpu:
            return
        cur = torch.cuda.current_stream(self.device)
        for s in [self.panel] + self.update:
            cur.wait_event(self.event(s))
