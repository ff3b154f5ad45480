"""Synchronous data parallelism: bucketed gradient all-reduce over RCCL, overlapped with backward.

This replaces the reference's parameter-server gradient path (dist-keras commit/pull
over TCP) with RCCL collectives over xGMI:

* Gradients live in ONE flat fp32 buffer (``models/params.py``).  Buckets are
  contiguous slices of it taken from the END (backward produces the last layers'
  gradients first), so an all-reduce needs no pack/unpack copies.
* Every layer fires a hook from its backward op as soon as its parameter gradients
  are final; when every parameter of a bucket is final the bucket's all-reduce is
  issued *from the compute stream* — RCCL's internal stream waits for exactly the
  kernels issued so far and then runs concurrently with the rest of the backward.
  Buckets launch strictly in index order on every rank (identical collective order,
  no deadlock even if hooks arrive in a slightly different order).
* Bucket size: xGMI is point-to-point (7 links x ~153 GB/s per MI355X); a ring
  all-reduce is bound by one link, so per-bucket latency alpha must be amortised by
  tens of MB.  Default 32 MB (override with ``bucket_mb`` / ``DDL_BUCKET_MB``).
* The 1/world averaging is folded into the optimizer kernel (``grad_scale``), so there
  is no separate scaling pass over the gradients.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from .comm import ProcessGroup


class DataParallel:
    def __init__(self, model, pg: ProcessGroup, bucket_mb: float | None = None, overlap: bool = True,
                 reduce_dtype: torch.dtype | None = None):
        self.model = model
        self.pg = pg
        self.overlap = overlap and pg.distributed
        if bucket_mb is None:
            bucket_mb = float(os.environ.get("DDL_BUCKET_MB", "32"))
        self.bucket_bytes = int(bucket_mb * (1 << 20))
        self.reduce_dtype = reduce_dtype
        model._ensure_placed()
        self.arena = model.arena
        self._build_buckets()
        self._works = []
        self.comm_time_hint = 0.0
        if self.overlap:
            self._install_hooks()

    # ---------------------------------------------------------------- buckets
    def _build_buckets(self):
        params = [p for p in self.arena.params if p.trainable]
        elems_per_bucket = max(self.bucket_bytes // 4, 1 << 14)
        buckets = []  # list of dict(start, end, params)
        cur = None
        for p in reversed(params):
            end = p.offset + (-(-p.numel // 64) * 64)
            if cur is None:
                cur = {"start": p.offset, "end": end, "params": [p]}
            else:
                cur["start"] = p.offset
                cur["params"].append(p)
            if cur["end"] - cur["start"] >= elems_per_bucket:
                buckets.append(cur)
                cur = None
        if cur is not None:
            buckets.append(cur)
        if buckets:
            buckets[0]["end"] = self.arena.numel  # include the alignment tail
            buckets[-1]["start"] = 0
        self.buckets = buckets
        self.bucket_of = {}
        for i, b in enumerate(buckets):
            for p in b["params"]:
                self.bucket_of[id(p)] = i

    def _install_hooks(self):
        for layer in self.model.all_layers():
            if layer._params:
                layer.grad_hook = (lambda L=layer: self._on_layer_grads(L))

    # ---------------------------------------------------------------- step protocol
    def _begin(self):
        self._pending = [len(b["params"]) for b in self.buckets]
        self._seen = set()
        self._ready = [False] * len(self.buckets)
        self._next = 0
        self._works = []

    def _on_layer_grads(self, layer):
        for p in layer._params:
            if id(p) in self._seen or id(p) not in self.bucket_of:
                continue
            self._seen.add(id(p))
            bi = self.bucket_of[id(p)]
            self._pending[bi] -= 1
            if self._pending[bi] == 0:
                self._ready[bi] = True
        self._launch_ready()

    def _launch_ready(self):
        while self._next < len(self.buckets) and self._ready[self._next]:
            self._launch(self._next)
            self._next += 1

    def _launch(self, i):
        b = self.buckets[i]
        view = self.arena.grad[b["start"] : b["end"]]
        self._works.append(self.pg.all_reduce_(view, async_op=True))

    def _finish(self):
        for i in range(self._next, len(self.buckets)):
            self._launch(i)
        self._next = len(self.buckets)
        for w in self._works:
            if w is not None:
                w.wait()
        self._works = []

    def sync_gradients(self, arena=None) -> float:
        """All-reduce every bucket (no overlap) — returns the averaging grad scale."""
        if self.pg.distributed:
            self._begin()
            self._finish()
        return 1.0 / self.pg.world_size

    # ---------------------------------------------------------------- public
    def broadcast_parameters(self, src: int = 0):
        """Rank ``src``'s weights to every replica (reference message M1: ship the model)."""
        if self.pg.distributed:
            self.pg.broadcast_(self.arena.master, src)
            self.arena.sync_compute()
            for layer in self.model.all_layers():
                for t in layer._states.values():
                    self.pg.broadcast_(t, src)

    def train_step(self, x, y, timer=None):
        """zero grads -> forward -> backward (bucket all-reduces overlap it) -> wait -> optimizer.

        ``timer``: optional :class:`utils.tracing.StepTimer` collecting per-phase GPU times;
        every phase is also a roctx range when tracing is on (``DDL_TRACE=1``)."""
        from ..ops.norm import reset_workspaces
        from ..utils.tracing import trace_range

        m = self.model
        phase = timer.phase if timer is not None else (lambda name: trace_range(name))
        with trace_range("train_step"):
            reset_workspaces(m.device)
            m.arena.zero_grad()
            if self.overlap:
                self._begin()
            with phase("forward"):
                loss = m.compute_loss(x, y, training=True)
            with phase("backward"):
                loss.backward()
            with phase("allreduce"):
                if self.overlap:
                    self._finish()
                elif self.pg.distributed:
                    self.sync_gradients()
            with phase("optimizer"):
                m.optimizer.step(grad_scale=1.0 / self.pg.world_size)
        return loss.detach()

    @property
    def grad_bytes(self) -> int:
        return self.arena.grad.numel() * self.arena.grad.element_size() if self.pg.distributed else 0

    def check_replicas(self, raise_on_mismatch: bool = True) -> bool:
        """Divergence detection: after a synchronous update every replica must
        hold identical weights.  Compares float64 (sum, sum-of-squares) checksums of the
        flat master buffer across ranks."""
        from ..utils.fault import replica_checksum

        if not self.pg.distributed:
            return True
        mine = replica_checksum(self.arena.master)
        allc = self.pg.all_gather_object(mine)
        ok = all(c == allc[0] for c in allc)
        if not ok and raise_on_mismatch:
            raise RuntimeError(f"data-parallel replicas diverged: checksums {allc}")
        return ok

    def all_reduce_flat_(self, t: torch.Tensor, average: bool = False):
        """All-reduce an arbitrary flat buffer in bucket-sized chunks (ADAG / DynSGD deltas)."""
        if not self.pg.distributed:
            return t
        step = max(self.bucket_bytes // t.element_size(), 1)
        works = [self.pg.all_reduce_(t[i : i + step], async_op=True) for i in range(0, t.numel(), step)]
        for w in works:
            w.wait()
        if average:
            t.div_(self.pg.world_size)
        return t
