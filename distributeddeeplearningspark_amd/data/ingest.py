"""Host -> HBM ingest: pinned host buffers streamed to the GPU on a side stream
(hipMemcpyAsync via ``Tensor.copy_(non_blocking=True)`` on a dedicated HIP stream),
overlapped with compute, followed by the fused normalise kernel
(``csrc/kernels/misc.hip: normalize_u8``: uint8 NHWC -> bf16, per-channel mean/std).

The next batch's copy is issued as soon as the current one is handed out, so the
PCIe transfer of batch i+1 runs under the forward/backward of batch i.
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops._native import C, use_native

IMAGENET_MEAN = (123.675, 116.28, 103.53)
IMAGENET_STD = (58.395, 57.12, 57.375)


class DeviceFeeder:
    """Double-buffered H2D feeder for (uint8 image batch, int64 labels) pairs."""

    def __init__(self, device, mean=IMAGENET_MEAN, std=IMAGENET_STD, out_dtype=torch.bfloat16):
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.stream = torch.cuda.Stream(self.device) if self.cuda else None
        self.mean = torch.tensor(mean, dtype=torch.float32, device=self.device)
        self.invstd = 1.0 / torch.tensor(std, dtype=torch.float32, device=self.device)
        self.out_dtype = out_dtype if self.cuda else torch.float32
        self._pending = None

    def submit(self, host_x: torch.Tensor, host_y: torch.Tensor):
        """Issue the async copy of a pinned batch (returns immediately)."""
        if not self.cuda:
            self._pending = (host_x, host_y, None)
            return
        with torch.cuda.stream(self.stream):
            dx = host_x.to(self.device, non_blocking=True)
            dy = host_y.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self._pending = (dx, dy, ev)

    def take(self):
        """Wait (on the compute stream, not the host) for the pending batch and normalise it."""
        dx, dy, ev = self._pending
        self._pending = None
        if ev is not None:
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(ev)
            dx.record_stream(cur)
            dy.record_stream(cur)
        return self.normalize(dx), dy

    def normalize(self, x_u8: torch.Tensor) -> torch.Tensor:
        Cc = x_u8.shape[-1]
        if use_native(x_u8):
            out = torch.empty(x_u8.shape, dtype=self.out_dtype, device=x_u8.device)
            C().normalize_u8(x_u8.contiguous(), out, self.mean[:Cc].contiguous(), self.invstd[:Cc].contiguous(), Cc, Cc)
            return out
        return ((x_u8.to(torch.float32) - self.mean[:Cc]) * self.invstd[:Cc]).to(self.out_dtype)


class SyntheticImageStream:
    """ImageNet-shaped synthetic batches (random uint8 pixels, random labels) in pinned
    host memory, cycled through the :class:`DeviceFeeder` exactly like a real loader."""

    def __init__(self, batch, image=224, num_classes=1000, channels=3, device="cuda", seed=0, n_buffers=4):
        self.device = torch.device(device)
        g = torch.Generator().manual_seed(seed)
        pin = self.device.type == "cuda"
        self.xs = [torch.randint(0, 256, (batch, image, image, channels), generator=g, dtype=torch.uint8)
                   for _ in range(n_buffers)]
        self.ys = [torch.randint(0, num_classes, (batch,), generator=g, dtype=torch.int64) for _ in range(n_buffers)]
        if pin:
            self.xs = [x.pin_memory() for x in self.xs]
            self.ys = [y.pin_memory() for y in self.ys]
        self.feeder = DeviceFeeder(self.device)
        self.i = 0
        self.feeder.submit(self.xs[0], self.ys[0])

    def next(self):
        x, y = self.feeder.take()
        self.i = (self.i + 1) % len(self.xs)
        self.feeder.submit(self.xs[self.i], self.ys[self.i])  # prefetch the next batch under this step
        return x, y


class ShardLoader:
    """Epoch iterator over a resident host shard, assembled by the native ``BatchLoader``
    (``csrc/runtime/loader.cpp``): a C++ thread gathers (optionally shuffled) rows into a
    ring of pinned buffers while the previous batch trains; each batch is copied to the
    device on a side stream.  Replaces the reference's per-row Python mini-batch assembly
    (``X = [row[features_col]]``, SURVEY §3.3 hot loop 3).

    Yields ``(x, y)`` device tensors; ``x`` is cast to ``x_dtype`` on the device.
    """

    def __init__(self, x: np.ndarray, y: np.ndarray | None, batch: int, device="cpu", shuffle=False, seed=0,
                 drop_last=True, n_buffers=4, threads=4, x_dtype=None):
        from ..ops._native import C

        self.x = torch.from_numpy(np.ascontiguousarray(x))
        self.y = None if y is None else torch.from_numpy(np.ascontiguousarray(y))
        self.batch, self.device = int(batch), torch.device(device)
        self.x_dtype = x_dtype
        self._impl = C().BatchLoader(self.x, self.y, self.batch, bool(shuffle), int(seed), bool(drop_last),
                                     int(threads))
        pin = self.device.type == "cuda"

        def buf(t):
            b = torch.empty((self.batch,) + tuple(t.shape[1:]), dtype=t.dtype)
            return b.pin_memory() if pin else b

        self._xb = [buf(self.x) for _ in range(n_buffers)]
        self._yb = [buf(self.y) for _ in range(n_buffers)] if self.y is not None else []
        self._impl.set_buffers(self._xb, self._yb)
        # the process-wide ingest side stream (one per device: co-located workers would otherwise
        # each claim a hardware queue per loader)
        if pin:
            from ..trainers import ingest_stream

            self._stream = ingest_stream(self.device)
        else:
            self._stream = None
        self.n_buffers = int(n_buffers)
        # pinned slots whose H2D copy may still be in flight: (slot, event), oldest first.  A slot
        # goes back to the C++ filler only once its copy event has completed, so the host runs up to
        # n_buffers - 2 batches ahead of the copies instead of synchronising on every batch.
        self._inflight: list = []
        self.epoch = 0

    def __len__(self):
        return self._impl.batches_per_epoch

    def _to_device(self, t, n):
        t = t[:n]
        if self._stream is None:
            return t.clone()
        with torch.cuda.stream(self._stream):
            d = t.to(self.device, non_blocking=True)
        # the compute stream reads d: the caching allocator must not hand its block to a later
        # side-stream copy before that read is done
        d.record_stream(torch.cuda.current_stream(self.device))
        return d

    def _reap(self, keep: int):
        """Release completed slots; block on the oldest copies until at most ``keep`` are in flight."""
        while self._inflight and (len(self._inflight) > keep or self._inflight[0][1].query()):
            slot, ev = self._inflight.pop(0)
            ev.synchronize()
            self._impl.release(slot)

    def __iter__(self):
        self._impl.start_epoch(self.epoch)
        self.epoch += 1
        keep = max(0, self.n_buffers - 2)  # the filler always owns >= 2 slots
        try:
            while True:
                self._reap(keep)
                slot, n = self._impl.next()
                if slot < 0:
                    return
                xd = self._to_device(self._xb[slot], n)
                yd = self._to_device(self._yb[slot], n) if self._yb else None
                if self._stream is not None:
                    ev = torch.cuda.Event()
                    ev.record(self._stream)
                    torch.cuda.current_stream(self.device).wait_event(ev)
                    self._inflight.append((slot, ev))
                else:
                    self._impl.release(slot)
                if self.x_dtype is not None and xd.is_floating_point():
                    xd = xd.to(self.x_dtype)
                yield xd, yd
        finally:
            self._reap(0)
