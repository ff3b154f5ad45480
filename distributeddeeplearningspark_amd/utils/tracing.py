"""Tracing and per-step timing.

* ``trace_range(name)`` — a roctx range (native, ``csrc/runtime/trace.cpp``) so that
  ``rocprofv3 --marker-trace`` shows step / fwd / bwd / allreduce / optimizer ranges next
  to the kernel trace; while a :class:`Tracer` is recording, the same ranges are also
  kept as host spans and dumped as a Chrome/Perfetto JSON trace.
* :class:`StepTimer` — GPU-side phase timing with HIP events on the compute stream and on
  the communication stream (allreduce time is measured where it runs).

Enabled by ``DDL_TRACE=1`` (roctx ranges only) or by an active :class:`Tracer`; otherwise
``trace_range`` is a no-op costing one attribute lookup.
"""
from __future__ import annotations

import contextlib
import json
import os
import time

import torch

from ..ops._native import has_native

_ACTIVE = {"on": os.environ.get("DDL_TRACE", "0") == "1", "tracer": None}


def _C():
    if not has_native():
        return None
    from ..ops._native import C

    return C()


@contextlib.contextmanager
def trace_range(name: str):
    if not _ACTIVE["on"]:
        yield
        return
    c = _C()
    t = _ACTIVE["tracer"]
    if c is not None:
        c.trace_push(name)
    elif t is not None:
        t._host_push(name)
    try:
        yield
    finally:
        if c is not None:
            c.trace_pop()
        elif t is not None:
            t._host_pop()


def mark(name: str):
    if _ACTIVE["on"] and _C() is not None:
        _C().trace_mark(name)


class Tracer:
    """Record host spans (and optional GPU event spans) and dump a Chrome trace JSON."""

    def __init__(self, rank: int = 0):
        self.rank = rank
        self.events = []
        self._stack = []
        self._gpu = []

    def __enter__(self):
        self.start()
        return self

    def __exit__(self, *exc):
        self.stop()

    def start(self):
        _ACTIVE["on"] = True
        _ACTIVE["tracer"] = self
        c = _C()
        if c is not None:
            c.trace_record(True)
        self._t0 = time.perf_counter_ns()
        return self

    def _host_push(self, name):
        self._stack.append((name, time.perf_counter_ns()))

    def _host_pop(self):
        if self._stack:
            name, t0 = self._stack.pop()
            self.events.append((name, t0, time.perf_counter_ns(), len(self._stack)))

    def gpu_span(self, name: str, start_evt, end_evt):
        """Register a GPU interval bracketed by two recorded torch.cuda.Events."""
        self._gpu.append((name, start_evt, end_evt))

    def stop(self):
        c = _C()
        if c is not None:
            self.events.extend(c.trace_collect())
            c.trace_record(False)
        _ACTIVE["tracer"] = None
        _ACTIVE["on"] = os.environ.get("DDL_TRACE", "0") == "1"

    def to_chrome(self) -> dict:
        evs = []
        base = min((e[1] for e in self.events), default=0)
        for name, t0, t1, depth in self.events:
            evs.append({"name": name, "ph": "X", "pid": self.rank, "tid": 0, "ts": (t0 - base) / 1e3,
                        "dur": (t1 - t0) / 1e3, "args": {"depth": depth}})
        if self._gpu:
            torch.cuda.synchronize()
            ref = self._gpu[0][1]
            for name, a, b in self._gpu:
                evs.append({"name": name, "ph": "X", "pid": self.rank, "tid": 1, "ts": ref.elapsed_time(a) * 1e3,
                            "dur": a.elapsed_time(b) * 1e3})
        return {"traceEvents": evs, "displayTimeUnit": "ms"}

    def dump(self, path: str):
        with open(path, "w") as f:
            json.dump(self.to_chrome(), f)
        return path


class StepTimer:
    """Per-phase GPU timing with HIP events: ``with timer.phase("fwd"): ...`` on the
    current stream, ``timer.phase("allreduce", stream=comm_stream)`` on another stream;
    ``timer.summary()`` synchronises once and returns milliseconds per phase."""

    def __init__(self, device=None):
        self.device = device
        self.enabled = torch.cuda.is_available() and (device is None or torch.device(device).type == "cuda")
        self._evs = []
        self._host = {}

    @contextlib.contextmanager
    def phase(self, name: str, stream=None):
        if not self.enabled:
            t0 = time.perf_counter()
            yield
            self._host[name] = self._host.get(name, 0.0) + (time.perf_counter() - t0) * 1e3
            return
        s = stream or torch.cuda.current_stream(self.device)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        with trace_range(name):
            yield
        b.record(s)
        self._evs.append((name, a, b))

    def summary(self, reset: bool = True) -> dict:
        out = dict(self._host)
        if self._evs:
            torch.cuda.synchronize(self.device)
            for name, a, b in self._evs:
                out[name] = out.get(name, 0.0) + a.elapsed_time(b)
        if reset:
            self._evs, self._host = [], {}
        return out
