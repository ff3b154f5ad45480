"""Synchronous data parallelism: bucketed gradient all-reduce over RCCL, overlapped with backward.

This replaces the reference's parameter-server gradient path (dist-keras commit/pull
over TCP; call sites ``ddl_mnist_aztk.py:216-219``) with RCCL
collectives over xGMI:

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
  tens of MB.  Measured, not assumed: on a GPU group of world > 1 the engine times a few
  all-reduces of 1 / 8 / 32 MB on the actual communicator at construction, fits
  t(S) = alpha + S / beta and takes the smallest power-of-two bucket with S / beta >= 5 alpha
  (:func:`bucket_policy`, 4-128 MB; rank 0's fit is broadcast so all ranks cut the same
  buckets; the fit is reported as ``DataParallel.calibration`` and in ``bench.py``'s JSON).
  ``bucket_mb`` / ``DDL_BUCKET_MB`` override it; CPU (gloo) groups use 32 MB.  The offline
  sweep is ``scripts/bench_allreduce.py``.  The bucket of the first layers is cut small
  (``DDL_TAIL_BUCKET_MB``, 4 MB): it is the one reduction that cannot overlap backward.
* ``reduce_dtype=torch.bfloat16`` (``DDL_REDUCE_DTYPE=bf16``): half the xGMI bytes, with
  ONE bf16 rounding of the cross-rank sum.  A ring all-reduce in bf16 would round every
  partial sum (N-1 bf16 additions per element at N=8, RCCL sums in the wire dtype); instead
  each bucket is cast to bf16 (HIP), exchanged with ONE all-to-all (rank r receives every
  rank's r-th chunk: point-to-point over all 7 xGMI links), summed locally in fp32 by a HIP
  kernel (``sum_rows_bf16``), and the summed chunks are all-gathered in bf16 and cast back
  into the fp32 arena — the same 2(N-1)/N wire bytes as a ring all-reduce.  The all-to-all
  of bucket i and the local sum + all-gather of bucket i-2 are pipelined through the hooks.
  ``DDL_BF16_ALGO=ring`` keeps the plain bf16 ring all-reduce (accuracy comparison:
  ``tests/test_ddp_cpu.py``); the default dtype stays fp32 for parity.
* The 1/world averaging is folded into the optimizer kernel (``grad_scale``), so there
  is no separate scaling pass over the gradients.
* Optimizer overlap: after backward, buckets are waited for in launch order and the fused
  optimizer updates each bucket's slice of the arena as soon as that bucket is reduced
  (``Optimizer.apply_range``), so the update of the early buckets runs under the reduction of
  the last one — the first layers' bucket (ResNet's stem, BERT's 94 MB word-embedding table,
  whose lookup gradient is only final at the very end of backward) is the one all-reduce
  that can never overlap backward, and it now overlaps the optimizer sweep instead.
* Timing (``timing=True``): HIP events on the compute stream bracket the part of the
  step that waits for communication (end of backward -> all buckets reduced), giving the
  *exposed* communication time; :meth:`measure_allreduce` times the full-gradient
  all-reduce on its own (``comm_ms`` in ``bench.py``'s JSON).
"""
from __future__ import annotations

import os

import torch

from .comm import ProcessGroup


def _reduce_dtype_from_env():
    v = os.environ.get("DDL_REDUCE_DTYPE", "fp32").lower()
    if v in ("bf16", "bfloat16"):
        return torch.bfloat16
    if v in ("fp32", "float32", "f32", ""):
        return torch.float32
    raise ValueError(f"DDL_REDUCE_DTYPE={v!r}: expected fp32 or bf16")


def all_reduce_flat(pg: ProcessGroup, t: torch.Tensor, bucket_bytes: int = 64 << 20, average: bool = False):
    """All-reduce an arbitrary flat buffer in bucket-sized chunks (ADAG / DynSGD deltas,
    model averaging).  Chunks are issued back to back (async) and waited together."""
    if not pg.distributed:
        return t
    step = max(int(bucket_bytes) // t.element_size(), 1)
    works = [pg.all_reduce_(t[i : i + step], async_op=True) for i in range(0, t.numel(), step)]
    for w in works:
        if w is not None:
            w.wait()
    if average:
        t.div_(pg.world_size)
    return t


def bucket_policy(alpha_s: float, beta_bps: float, k: float = 5.0, lo_mb: float = 4.0, hi_mb: float = 128.0) -> float:
    """Bucket size (MB) for an all-reduce cost t(S) = alpha + S / beta: the smallest bucket whose
    bandwidth term is k x the per-call latency, S = k * alpha * beta, rounded up to a power of two and
    clamped to [lo, hi] MB.  Small buckets overlap backward at a finer grain; below this size the per-call
    latency of the collective (RCCL kernel launch + ring setup over the point-to-point xGMI links)
    dominates the bytes it moves."""
    import math

    if not (alpha_s > 0 and beta_bps > 0):
        return 32.0
    mb = k * alpha_s * beta_bps / (1 << 20)
    mb = 2.0 ** math.ceil(math.log2(max(mb, 1e-3)))
    return float(min(max(mb, lo_mb), hi_mb))


_CALIB: dict = {}


def calibrate_allreduce(pg: ProcessGroup, device, sizes_mb=(1, 8, 32), iters: int = 3):
    """Time fp32 all-reduces of ``sizes_mb`` on this group and fit t(S) = alpha + S / beta (least squares over
    the medians); rank 0's fit is broadcast so every rank cuts identical buckets.  Runs once per group on GPU
    (RCCL) groups of world > 1 only — CPU gloo groups, forced world-1 groups and co-located host-staged
    groups keep the 32 MB default.  Returns {"alpha_us", "gbps", "bucket_mb", "points"} or None."""
    import time

    if not pg.distributed or pg.world_size < 2 or pg.host_staged or device is None or torch.device(device).type != "cuda":
        return None
    key = (pg.world_size, pg.rank, str(device), id(pg.group))
    if key in _CALIB:
        return _CALIB[key]
    pts = []
    for mb in sizes_mb:
        t = torch.ones((int(mb) << 20) // 4, dtype=torch.float32, device=device)
        pg.all_reduce_(t)  # warm-up (communicator / channel setup)
        torch.cuda.synchronize(device)
        ts = []
        for _ in range(iters):
            pg.barrier()
            t0 = time.perf_counter()
            pg.all_reduce_(t)
            torch.cuda.synchronize(device)
            ts.append(time.perf_counter() - t0)
        ts.sort()
        pts.append((float(mb) * (1 << 20), ts[len(ts) // 2]))
    n = len(pts)
    sx, sy = sum(x for x, _ in pts), sum(y for _, y in pts)
    sxx, sxy = sum(x * x for x, _ in pts), sum(x * y for x, y in pts)
    slope = (n * sxy - sx * sy) / max(n * sxx - sx * sx, 1e-30)
    alpha = max((sy - slope * sx) / n, 1e-6)
    beta = 1.0 / slope if slope > 0 else 1e12
    res = {"alpha_us": round(alpha * 1e6, 2), "gbps": round(beta / 1e9, 2), "bucket_mb": bucket_policy(alpha, beta),
           "points": [(int(x) >> 20, round(y * 1e3, 4)) for x, y in pts]}
    res = pg.broadcast_object(res)
    _CALIB[key] = res
    return res


def _bf16_algo() -> str:
    v = os.environ.get("DDL_BF16_ALGO", "a2a").lower()
    if v not in ("a2a", "ring"):
        raise ValueError(f"DDL_BF16_ALGO={v!r}: expected a2a or ring")
    return v


def _sum_rows_bf16(x: torch.Tensor, y: torch.Tensor):
    """y = bf16(sum over rows of x) with an fp32 accumulator (HIP on the GPU)."""
    from ..ops._native import C, use_native

    if use_native(x):
        C().sum_rows_bf16(x, y)
    else:
        y.copy_(x.float().sum(0))


class _A2ABucket:
    """bf16-wire reduction of one bucket: cast -> all-to-all -> fp32 local sum -> all-gather -> cast back.
    ``start`` / ``middle`` / ``finish`` are the three collective phases; each collective is async and
    the compute stream waits on it (device-side) only at the next phase."""

    def __init__(self, view: torch.Tensor, pg: ProcessGroup):
        import torch.distributed as dist

        self.dist = dist
        self.view, self.pg = view, pg
        N = pg.world_size
        L = view.numel()
        chunk = -(-L // N)  # ceil(L / N) elements per rank, rounded up to 64 (16-B rows)
        chunk = -(-chunk // 64) * 64
        self.L, self.N, self.chunk = L, N, chunk
        dev = view.device
        self.send = torch.zeros(N * chunk, dtype=torch.bfloat16, device=dev)  # pad tail stays zero
        self.recv = torch.empty(N * chunk, dtype=torch.bfloat16, device=dev)
        self.gath = torch.empty(N * chunk, dtype=torch.bfloat16, device=dev)
        self.mine = torch.empty(chunk, dtype=torch.bfloat16, device=dev)
        self.w1 = self.w2 = None
        self.phase = 0

    def start(self):
        _cast(self.view, self.send[: self.L])
        self.w1 = self.dist.all_to_all_single(self.recv, self.send, group=self.pg.group, async_op=True)
        self.phase = 1

    def middle(self):
        if self.phase != 1:
            return
        self.w1.wait()
        _sum_rows_bf16(self.recv.view(self.N, self.chunk), self.mine)
        self.w2 = self.dist.all_gather_into_tensor(self.gath, self.mine, group=self.pg.group, async_op=True)
        self.phase = 2

    def finish(self):
        self.middle()
        if self.phase != 2:
            return
        self.w2.wait()
        _cast(self.gath[: self.L], self.view)
        self.phase = 3


def _cast(src: torch.Tensor, dst: torch.Tensor):
    """fp32 <-> bf16 over flat slices: HIP kernels on the GPU, torch on the CPU."""
    from ..ops._native import C, use_native

    if use_native(src):
        if src.dtype == torch.float32:
            C().cast_f32_bf16(src, dst)
        else:
            C().cast_bf16_f32(src, dst)
    else:
        dst.copy_(src)


class DataParallel:
    def __init__(self, model, pg: ProcessGroup, bucket_mb: float | None = None, overlap: bool = True,
                 reduce_dtype: torch.dtype | None = None, timing: bool = False):
        self.model = model
        self.pg = pg
        self.overlap = overlap and pg.distributed
        self.calibration = None
        if bucket_mb is None:
            env = os.environ.get("DDL_BUCKET_MB", "auto")
            from ..ops import determinism

            if env == "auto" and determinism.enabled():
                # reproducible multi-rank runs need fixed bucket boundaries (a timing-based size can
                # change RCCL's chunking, and with it the summation order, from run to run)
                bucket_mb = 32.0
            elif env == "auto":
                # measured on THIS group (RCCL over xGMI on a GPU node): see bucket_policy / calibrate_allreduce
                self.calibration = calibrate_allreduce(pg, model.arena.grad.device if model.arena is not None else None)
                bucket_mb = self.calibration["bucket_mb"] if self.calibration else 32.0
            else:
                bucket_mb = float(env)
        self.bucket_mb = float(bucket_mb)
        self.bucket_bytes = int(bucket_mb * (1 << 20))
        self.reduce_dtype = reduce_dtype if reduce_dtype is not None else _reduce_dtype_from_env()
        if self.reduce_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError(f"reduce_dtype {self.reduce_dtype}: expected torch.float32 or torch.bfloat16")
        model._ensure_placed()
        self.arena = model.arena
        self._red = None  # bf16 mirror of the gradient arena (ring algorithm, allocated once)
        self.bf16_algo = None
        if self.reduce_dtype == torch.bfloat16 and pg.distributed:
            # all-to-all + local fp32 sum; host-staged (co-located gloo) groups keep the ring
            self.bf16_algo = "ring" if pg.host_staged else _bf16_algo()
            if self.bf16_algo == "ring":
                self._red = torch.zeros(self.arena.numel, dtype=torch.bfloat16, device=self.arena.grad.device)
        self._build_buckets()
        self._a2a = None
        if self.bf16_algo == "a2a":
            self._a2a = [_A2ABucket(self.arena.grad[b["start"]: b["end"]], pg) for b in self.buckets]
        self._works = []
        # optimizer overlap (see module doc): each bucket's arena slice is updated once it is reduced
        self.overlap_optimizer = os.environ.get("DDL_OVERLAP_OPTIMIZER", "1") != "0"
        self.timing = bool(timing) and self.arena.grad.is_cuda
        self._events = []  # (backward done, comm done) per timed step
        if self.overlap:
            self._install_hooks()

    # ---------------------------------------------------------------- buckets
    def _build_buckets(self):
        params = [p for p in self.arena.params if p.trainable]
        # bucket size is counted in WIRE bytes, so a bf16 reduce packs twice the elements
        wire = 2 if self.bf16_algo is not None else 4
        elems_per_bucket = max(self.bucket_bytes // wire, 256)
        # The bucket holding the FIRST layers launches only after the whole backward is done, so
        # its all-reduce is never hidden: it is cut from the front of the arena at a small size
        # (DDL_TAIL_BUCKET_MB, default min(4 MB, bucket)), the rest in full-size buckets.  With
        # buckets cut from the end instead, ResNet-50's last 32 MB bucket spanned stage 3 down to
        # the stem and its whole reduction waited for the stem's gradients.
        tail_mb = float(os.environ.get("DDL_TAIL_BUCKET_MB", min(4.0, self.bucket_mb)))
        cap = max(int(tail_mb * (1 << 20)) // wire, 256)
        buckets = []  # built front -> back, reversed below: index 0 = end of the arena
        cur = None
        for p in params:
            end = p.offset + (-(-p.snumel // 64) * 64)
            if cur is None:
                cur = {"start": p.offset, "end": end, "params": [p]}
            else:
                cur["end"] = end
                cur["params"].append(p)
            if cur["end"] - cur["start"] >= cap:
                buckets.append(cur)
                cur = None
                cap = elems_per_bucket
        if cur is not None:
            buckets.append(cur)
        buckets.reverse()
        for b in buckets:
            b["params"].reverse()
        if buckets:
            buckets[0]["end"] = self.arena.numel  # include the alignment tail
            buckets[-1]["start"] = 0
        self.buckets = buckets
        # optimizer ranges: a partition of [0, numel) in bucket launch order (bucket i owns
        # [start_i, start_{i-1}), so gaps of non-trainable parameters are covered too)
        prev = self.arena.numel
        for b in buckets:
            b["opt_range"] = (b["start"], prev)
            prev = b["start"]
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
        from ..ops.streams import on_grad_stream

        # launched from the weight-gradient side stream (after it has waited for the compute
        # stream): RCCL then orders the bucket after its side-stream weight gradients AND the
        # compute-stream BatchNorm / bias gradients (ops/streams.py)
        with on_grad_stream(self.arena.grad.device):
            self._launch_on_stream(i)

    def _launch_on_stream(self, i):
        b = self.buckets[i]
        view = self.arena.grad[b["start"] : b["end"]]
        if self._a2a is not None:
            # second phase (local sum + all-gather) of the bucket launched two before: a fixed
            # schedule, so every rank issues the collectives in the same order (a completion-driven
            # choice would differ between ranks and deadlock)
            if i >= 2:
                self._a2a[i - 2].middle()
            self._a2a[i].start()
            self._works.append(None)
            return
        if self._red is not None:
            red = self._red[b["start"] : b["end"]]
            _cast(view, red)  # on the compute stream: ordered after the bucket's last grad kernel
            view = red
        self._works.append(self.pg.all_reduce_(view, async_op=True))

    def _wait_bucket(self, i):
        """Compute stream waits (device-side) until bucket i is fully reduced into the fp32 arena."""
        if self._a2a is not None:
            self._a2a[i].finish()
            return
        w = self._works[i]
        if w is not None:
            w.wait()
        if self._red is not None:
            b = self.buckets[i]
            _cast(self._red[b["start"] : b["end"]], self.arena.grad[b["start"] : b["end"]])

    def _finish(self, optimizer=None, grad_scale: float = 1.0, reduced_event=None) -> bool:
        """Launch what is left, then wait bucket by bucket.  With ``optimizer`` (ranged-capable),
        each bucket's arena slice is updated right after its wait; returns True if it stepped.
        ``reduced_event`` is recorded on the compute stream once the LAST bucket is reduced."""
        from ..ops.streams import join

        for i in range(self._next, len(self.buckets)):
            self._launch(i)
        self._next = len(self.buckets)
        join(self.arena.grad.device)  # the updates below read every weight gradient
        ranged = optimizer is not None and optimizer.ranged_ok and self.overlap_optimizer
        gs = optimizer.begin_step(grad_scale) if ranged else None
        for i, b in enumerate(self.buckets):
            self._wait_bucket(i)
            if reduced_event is not None and i == len(self.buckets) - 1:
                reduced_event.record()
            if ranged:
                optimizer.apply_range(*b["opt_range"], gs)
        self._works = []
        return ranged

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
            reset_workspaces(m.device, extra=m.arena.zero_grad(defer=True))  # one zeroing launch
            if self.overlap:
                self._begin()
            from ..ops import derived

            derived.begin_step(m)  # weight-derived filters: one launch per step (ops/derived.py)
            try:
                with phase("forward"):
                    loss = m.compute_loss(x, y, training=True)
                with phase("backward"):
                    m.backward_unit(loss)
            finally:
                derived.end_step()
            ev = None
            if self.timing and self.pg.distributed:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            stepped = False
            with phase("allreduce"):
                if self.pg.distributed:
                    if not self.overlap:
                        self._begin()
                    # the optimizer rides bucket by bucket behind the waits (a per-phase timer keeps
                    # the two apart, so its phase GPU times stay attributable).  Exposed comm = end of
                    # backward -> last bucket reduced; with the ranged optimizer that window also
                    # holds the update of every earlier bucket, so it is an upper bound.
                    stepped = self._finish(m.optimizer if timer is None else None, 1.0 / self.pg.world_size,
                                           reduced_event=None if ev is None else ev[1])
            if ev is not None:
                if not self.pg.distributed or not self.buckets:
                    ev[1].record()
                self._events.append(ev)
            if not stepped:
                with phase("optimizer"):
                    m.optimizer.step(grad_scale=1.0 / self.pg.world_size)
        return loss.detach()

    def exposed_comm_ms(self, reset: bool = True) -> float | None:
        """Mean GPU time per timed step between the end of backward and the moment every
        bucket is reduced (the communication NOT hidden behind backward).  Call after a
        device synchronize."""
        if not self._events:
            return None
        v = sum(a.elapsed_time(b) for a, b in self._events) / len(self._events)
        if reset:
            self._events = []
        return v

    def measure_allreduce(self, iters: int = 10, warmup: int = 2) -> float | None:
        """Milliseconds for one full-gradient all-reduce (every bucket, same dtype / bucket
        plan as the step), measured alone on the compute stream.  Leaves the gradient
        arena scaled by world**(iters+warmup): call it outside training, then zero grads."""
        if not self.pg.distributed or not self.arena.grad.is_cuda:
            return None
        for _ in range(warmup):
            self.sync_gradients()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            self.sync_gradients()
        b.record()
        b.synchronize()
        self.arena.zero_grad()
        return a.elapsed_time(b) / iters

    @property
    def grad_bytes(self) -> int:
        """Bytes each rank puts through the all-reduce per step."""
        if not self.pg.distributed:
            return 0
        return self.arena.grad.numel() * (2 if self.bf16_algo is not None else 4)

    def bucket_report(self) -> list[dict]:
        """Launch-order bucket table: index, MB on the wire, first/last parameter names."""
        wire = 2 if self.bf16_algo is not None else 4
        return [{"index": i, "mb": (b["end"] - b["start"]) * wire / (1 << 20), "params": len(b["params"]),
                 "first": b["params"][0].name, "last": b["params"][-1].name} for i, b in enumerate(self.buckets)]

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
        """All-reduce an arbitrary flat buffer in this engine's bucket size."""
        return all_reduce_flat(self.pg, t, self.bucket_bytes, average)
