"""Tracing (SLATE `trace::Trace`, `include/slate/internal/Trace.hh:18-112`,
`src/auxiliary/Trace.cc:176-644`).

* ``trace_block(name)`` -- RAII-style span: host wall time recorded into the
  native :class:`_host.TraceRecorder`; when on a GPU and device timing is
  enabled, a pair of HIP events on the current stream also records the
  span's *device* time (SLATE only has host spans that include queue syncs).
* ``Trace.on() / off() / finish(path)`` -- gather events of all ranks to
  rank 0 and write a Chrome-trace JSON (chrome://tracing / Perfetto) and an
  SVG timeline in the spirit of SLATE's ``trace_<time>.svg``.
"""
from __future__ import annotations

import contextlib
import json
import os
import threading
import time

import torch

from . import watchdog as _wd

from .. import _native

_rec = _native._host.TraceRecorder()
_dev_events = []
_nest = threading.local()
_device_timing = False

# fixed colour map keyed by routine name prefix (Trace.cc:187-255 analogue)
COLORS = {
    "gemm": "#4a90d9", "herk": "#2e7d32", "trsm": "#f9a825", "potrf": "#c62828",
    "getrf": "#6a1b9a", "geqrf": "#00838f", "bcast": "#ef6c00", "panel": "#ad1457",
    "trailing": "#1565c0", "laswp": "#8d6e63", "comm": "#ef6c00",
}


class Trace:
    @staticmethod
    def on(device_timing=False):
        global _device_timing
        _device_timing = bool(device_timing) and torch.cuda.is_available()
        _rec.clear()
        _dev_events.clear()
        _rec.on()

    @staticmethod
    def off():
        _rec.off()

    @staticmethod
    def is_on():
        return _rec.is_on()

    @staticmethod
    def events():
        t0 = _rec.t0()
        ev = [dict(name=n, start=(a - t0), stop=(b - t0), lane=int(l), nest=int(k), kind="host")
              for (n, a, b, l, k) in _rec.events()]
        if _dev_events:
            torch.cuda.synchronize()
            for (name, e0, e1, host_start) in _dev_events:
                dt = e0.elapsed_time(e1) * 1e-3
                ev.append(dict(name=name, start=host_start - t0, stop=host_start - t0 + dt, lane=1000,
                               nest=0, kind="device"))
        return ev

    @staticmethod
    def finish(path=None, comm=None):
        """Gather all ranks' events and write <path>.json and <path>.svg on rank 0."""
        from ..parallel.comm import world
        comm = comm or world()
        evs = Trace.events()
        allev = [evs]
        if comm.size > 1:
            import torch.distributed as dist
            out = [None] * comm.size
            dist.all_gather_object(out, evs)
            allev = out
        Trace.off()
        if comm.rank != 0:
            return None
        path = path or f"trace_{int(time.time())}"
        chrome = []
        for r, evs_r in enumerate(allev):
            for e in evs_r:
                chrome.append(dict(name=e["name"], ph="X", ts=e["start"] * 1e6, dur=(e["stop"] - e["start"]) * 1e6,
                                   pid=r, tid=e["lane"], cat=e["kind"]))
        with open(path + ".json", "w") as f:
            json.dump({"traceEvents": chrome}, f)
        _write_svg(path + ".svg", allev)
        return path


def _color(name):
    for k, v in COLORS.items():
        if k in name:
            return v
    return "#9e9e9e"


def _write_svg(path, allev, width=1600, row_h=20):
    rows = []
    for r, evs in enumerate(allev):
        lanes = sorted({e["lane"] for e in evs})
        for l in lanes:
            rows.append((r, l, [e for e in evs if e["lane"] == l]))
    tmax = max([e["stop"] for evs in allev for e in evs] + [1e-9])
    h = row_h * (len(rows) + 2)
    out = [f'<svg xmlns="http://www.w3.org/2000/svg" width="{width + 120}" height="{h}">',
           '<!-- slate_amd trace: one row per (rank, thread/stream) -->']
    for i, (r, l, evs) in enumerate(rows):
        y = row_h * (i + 1)
        out.append(f'<text x="2" y="{y + 14}" font-size="11">r{r}:{"dev" if l == 1000 else l}</text>')
        for e in evs:
            x = 110 + width * e["start"] / tmax
            w = max(0.5, width * (e["stop"] - e["start"]) / tmax)
            out.append(f'<rect x="{x:.2f}" y="{y}" width="{w:.2f}" height="{row_h - 2}" '
                       f'fill="{_color(e["name"])}"><title>{e["name"]} {1e3 * (e["stop"] - e["start"]):.3f} ms'
                       f'</title></rect>')
    out.append("</svg>")
    with open(path, "w") as f:
        f.write("\n".join(out))


@contextlib.contextmanager
def trace_block(name):
    # every traced region is also a library region for the watchdog: it
    # checks staleness only while some driver is running, and every region
    # entry / exit is a heartbeat
    _wd.enter(name)
    try:
        if not _rec.is_on():
            yield
            return
        yield from _traced(name)
    finally:
        _wd.leave(name)


def _traced(name):
    depth = getattr(_nest, "d", 0)
    _nest.d = depth + 1
    e0 = None
    if _device_timing and torch.cuda.is_available():
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
    t0 = _rec.now()
    try:
        yield
    finally:
        t1 = _rec.now()
        _rec.add(name, t0, t1, _rec.thread_lane(), depth)
        if e0 is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            _dev_events.append((name, e0, e1, t0))
        _nest.d = depth
