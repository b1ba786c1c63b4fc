"""Per-phase timers (`slate::timers`, include/slate/slate.hh:35-38;
filled by drivers e.g. "posv::potrf", "heev::he2hb").

``timer(name)`` measures host wall time; on a GPU it brackets the span with
HIP events so the recorded value is DEVICE time once the stream drains
(``timers()`` resolves pending events lazily)."""
from __future__ import annotations

import contextlib
import time

import torch

_timers = {}
_pending = []


def timers() -> dict:
    if _pending:
        torch.cuda.synchronize()
        for name, e0, e1 in _pending:
            _timers[name] = _timers.get(name, 0.0) + e0.elapsed_time(e1) * 1e-3
        _pending.clear()
    return dict(_timers)


def clear():
    _timers.clear()
    _pending.clear()


@contextlib.contextmanager
def timer(name, device=None):
    gpu = torch.cuda.is_available() if device is None else device
    if gpu:
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        try:
            yield
        finally:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            _pending.append((name, e0, e1))
    else:
        t0 = time.perf_counter()
        try:
            yield
        finally:
            _timers[name] = _timers.get(name, 0.0) + time.perf_counter() - t0


class Timer:
    """SLATE `Timer` (util.hh): wall-clock stopwatch."""

    def __init__(self):
        self.t0 = time.perf_counter()

    def stop(self):
        return time.perf_counter() - self.t0
