"""Communication / progress watchdog (SURVEY §5.3 failure detection).

The reference has no watchdog: an MPI rank that dies or deadlocks hangs the
job.  On MI355X the collectives are RCCL kernels enqueued on HIP streams, so
a lost peer shows up as a stream that never drains.  Two layers:

* ``comm.init`` passes an explicit collective timeout to
  ``torch.distributed`` (``SLATE_AMD_COMM_TIMEOUT`` seconds, default 600):
  RCCL's own watchdog then aborts a collective stuck past it and the
  process exits instead of spinning forever.
* :class:`Watchdog` -- a host thread that watches heartbeats.  Every
  ``Comm`` collective and every driver step calls :func:`beat` with a tag
  (``"bcast"``, ``"potrf step 17"``); if no beat arrives for ``timeout``
  seconds while the watchdog is armed it reports the rank, the last tag and
  its age, dumps every Python thread's stack (``faulthandler``), calls the
  user callback and, when ``abort`` is set, ends the process with exit
  status 3 so the launcher (torchrun) tears the job down.

``SLATE_AMD_WATCHDOG=<seconds>`` arms it from ``comm.init``.

Staleness is only checked while the process is INSIDE the library: every
driver region (``trace_block``) calls :func:`enter` / :func:`leave`, which
keep a depth count and beat.  Time the application spends outside
slate_amd -- its own compute, I/O, waiting for input -- never fires the
watchdog.  Inside, the limit must exceed the longest single phase that
cannot beat (one GPU call such as the bulge chase of heev, a few seconds at
n = 16384); the default collective timeout is 600 s.
"""
from __future__ import annotations

import faulthandler
import os
import sys
import threading
import time
from typing import Callable, Optional

_state = {"tag": "start", "t": time.monotonic(), "n": 0}
_lock = threading.Lock()
_active: Optional["Watchdog"] = None


def beat(tag: str = "") -> None:
    """Record progress (cheap: one monotonic clock read and two stores)."""
    _state["t"] = time.monotonic()
    _state["tag"] = tag
    _state["n"] += 1


_depth = [0]          # library regions open in this PROCESS (all threads; under _lock)


def enter(tag: str = "") -> None:
    """Entering a library region (nestable, thread-safe)."""
    with _lock:
        _depth[0] += 1
    beat(tag)


def leave(tag: str = "") -> None:
    with _lock:
        _depth[0] = max(0, _depth[0] - 1)
    beat(tag)


def watched(tag: str):
    """Decorator: the call is a library region (enter / leave around it).
    Every Comm collective and point-to-point call carries it, so a peer lost
    in a barrier or all-reduce OUTSIDE any driver -- bench's timing
    barriers, finalize, user-level comm calls -- still trips the watchdog
    (ADVICE r3)."""
    import functools

    def deco(fn):
        @functools.wraps(fn)
        def wrapped(*a, **k):
            enter(tag)
            try:
                return fn(*a, **k)
            finally:
                leave(tag)
        return wrapped
    return deco


def inside() -> bool:
    return _depth[0] > 0


def last_beat():
    """(tag, seconds since, number of beats)."""
    return _state["tag"], time.monotonic() - _state["t"], _state["n"]


class Watchdog:
    def __init__(self, timeout: float, abort: bool = True,
                 callback: Optional[Callable[[dict], None]] = None, poll: Optional[float] = None):
        self.timeout = float(timeout)
        self.abort = abort
        self.callback = callback
        self.poll = poll if poll is not None else max(0.05, min(5.0, self.timeout / 4))
        self.fired = None
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, name="slate_amd-watchdog", daemon=True)

    def start(self) -> "Watchdog":
        global _active
        beat("watchdog armed")
        self._thread.start()
        _active = self
        return self

    def stop(self) -> None:
        global _active
        self._stop.set()
        if self._thread.is_alive() and threading.current_thread() is not self._thread:
            self._thread.join(timeout=2 * self.poll + 1)
        if _active is self:
            _active = None

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
        return False

    def _report(self, tag, age, n) -> dict:
        rank = os.environ.get("RANK", "0")
        info = {"rank": int(rank), "tag": tag, "age_s": age, "beats": n, "timeout_s": self.timeout}
        print(f"[slate_amd watchdog] rank {rank}: no progress for {age:.1f} s "
              f"(limit {self.timeout:.1f} s); last step: {tag!r} after {n} beats",
              file=sys.stderr, flush=True)
        try:
            faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
        except Exception:  # noqa: BLE001 -- stderr may not have a fileno under capture
            pass
        return info

    def _run(self):
        while not self._stop.wait(self.poll):
            tag, age, n = last_beat()
            if age <= self.timeout or not inside():
                continue
            self.fired = self._report(tag, age, n)
            if self.callback is not None:
                self.callback(self.fired)
            if self.abort:
                sys.stderr.flush()
                os._exit(3)
            return


def active() -> Optional[Watchdog]:
    return _active


def from_env() -> Optional[Watchdog]:
    """Arm a watchdog from SLATE_AMD_WATCHDOG=<seconds> (once per process)."""
    v = os.environ.get("SLATE_AMD_WATCHDOG")
    if not v or _active is not None:
        return _active
    return Watchdog(float(v), abort=os.environ.get("SLATE_AMD_WATCHDOG_ABORT", "1") != "0").start()
