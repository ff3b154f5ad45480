"""Graph-captured training step: ONE hipGraph replay per mini-batch.

The reference's own workloads (MNIST CNN at batch 16, GRU/LSTM regressors at batch 32,
``ddl_mnist_aztk.py:217``, ``ddl_nyiso_aztk.py:86-88``) are tiny: a training step is a
few dozen kernels of a few microseconds each, so an eager step is bound by host-side
launch and autograd overhead, not by the GPU.  On MI355X the fix is a HIP graph (the
tracing-compiler-free way to remove launch cost): the whole step — zero grads, forward,
loss, backward into the flat gradient arena, fused optimizer update — is captured once
with static input/target buffers and then replayed.  Per mini-batch the host issues two
device-to-device copies into the static buffers and one ``hipGraphLaunch``; the loss
stays on the GPU until the caller asks for it.

Graph-safety of the captured work:
* every kernel launches on the current (capturing) stream (``csrc/*_bindings.cpp``);
* statistics workspaces come from a pool whose layout is fixed after the first step;
* the Adam step counter lives on the device (``Optimizer.enable_device_step``), so the
  bias corrections advance on every replay;
* Dropout layers' counter-hash kernels mix a device step counter into their capture-time seeds and the
  captured step ticks it, so every replay draws fresh masks (``ops/act.py dropout_step_counter``).
Models that need host-side per-step state (gradient clipping by global norm, BERT's step-seeded
dropout hashes) report ``graph_capturable = False`` and run eagerly.

Used by the dist-keras workers (``trainers.py``) whenever a worker trains on a GPU.
"""
from __future__ import annotations

import contextlib
import gc
import os

import torch


@contextlib.contextmanager
def graph_capture(g, stream):
    """``torch.cuda.graph(g, stream=stream)`` with Python's cyclic garbage collector off for the capture: a
    collection that starts inside a capture runs the destructors of unrelated garbage (events, graphs and
    streams of finished models), and their HIP calls are illegal while a stream captures — the process
    aborts (seen once in the GPU suite, a co-located replica capture collecting mid-window)."""
    was = gc.isenabled()
    gc.disable()  # no gc.collect() first: a full collection per capture cost the NYISO replica groups ~50 ms
    try:
        with torch.cuda.graph(g, stream=stream):
            yield
    finally:
        if was:
            gc.enable()


def graphs_enabled() -> bool:
    return os.environ.get("DDL_GRAPHS", "1") != "0"


def _uses_dropout(model) -> bool:
    from .layers import Dropout

    return any(isinstance(l, Dropout) and l.rate > 0 for l in model.all_layers())


class CompiledTrainStep:
    """``step(x, y) -> loss`` (0-d fp32 GPU tensor, overwritten by the next call).

    The first ``warmup`` calls run eagerly (they are real training steps: they also
    settle lazily-allocated workspaces); the next call captures and replays.  Shapes and
    dtypes of ``x``/``y`` must stay fixed (the dist-keras workers drop a trailing partial
    batch, so they do)."""

    def __init__(self, model, warmup: int = 2):
        self.model = model
        self.warmup = int(warmup)
        self.calls = 0
        self.graph = None
        self.static_x = self.static_y = self.static_loss = None
        self.captured = False
        self.fallback_reason = None
        self.enabled = self._can_capture()

    def _can_capture(self):
        m = self.model
        if not graphs_enabled():
            self.fallback_reason = "DDL_GRAPHS=0"
            return False
        if m.device.type != "cuda":
            self.fallback_reason = "not on a GPU"
            return False
        if not getattr(m, "graph_capturable", True):
            self.fallback_reason = f"{type(m).__name__} keeps host-side per-step state"
            return False
        if getattr(m.optimizer, "clipnorm", None) is not None:
            self.fallback_reason = "clipnorm reads the gradient norm on the host"
            return False
        return True

    # ---------------------------------------------------------------- eager step
    def _eager(self, x, y):
        m = self.model
        loss = m.backward_step(x, y)
        m.optimizer.step(1.0)
        return loss.detach().float()

    def _capture(self, x, y):
        m = self.model
        m.optimizer.enable_device_step()
        self.static_x = x.clone()
        self.static_y = y.clone()
        g = torch.cuda.CUDAGraph()  # a hipGraph on ROCm
        # capture on a side stream (required by the stream-capture API), then join
        s = torch.cuda.Stream(device=m.device)
        s.wait_stream(torch.cuda.current_stream(m.device))
        with torch.cuda.stream(s):
            with graph_capture(g, s):
                loss = m.backward_step(self.static_x, self.static_y)
                m.optimizer.captured_update(1.0)
                self.static_loss = loss.detach().float()
                if _uses_dropout(m):  # fresh dropout masks on every replay (ops/act.py)
                    from ..ops.act import tick_dropout_step

                    tick_dropout_step(m.device)
        torch.cuda.current_stream(m.device).wait_stream(s)
        from ..ops.norm import _POOL

        # the replayed kernels address these buffers: keep them alive even if the
        # (global) statistics pool is later regrown by another model
        self._keep = [b for b in _POOL.buf.values()]
        self.graph = g
        self.captured = True

    def __call__(self, x, y):
        m = self.model
        self.calls += 1
        if not self.enabled or self.calls <= self.warmup:
            return self._eager(x, y)
        if self.graph is None:
            try:
                self._capture(x, y)
            except Exception as e:  # capture is an optimisation: fall back loudly but keep training
                self.enabled, self.fallback_reason = False, f"capture failed: {type(e).__name__}: {e}"
                if os.environ.get("DDL_GRAPHS_STRICT") == "1":
                    raise
                print(f"[ddl] hipGraph capture disabled: {self.fallback_reason}", flush=True)
                torch.cuda.synchronize(m.device)
                return self._eager(x, y)
        else:
            self.static_x.copy_(x, non_blocking=True)
            self.static_y.copy_(y, non_blocking=True)
        self.graph.replay()
        m.optimizer.iterations += 1  # host mirror of the device step counter
        return self.static_loss
