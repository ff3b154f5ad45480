"""Flat parameter arena: every trainable tensor of a model lives in ONE contiguous
fp32 master buffer, ONE compute-dtype copy (bf16 on MI355X) and ONE fp32 gradient
buffer.

Why: the optimizer is a single launch over the flat buffer, the data-parallel
all-reduce works on contiguous bucket slices of the gradient buffer without any
packing copies (RCCL sees 16-MB-class messages, not hundreds of small tensors), and
checkpoints / the reference's ``get_weights()`` are slices of one buffer.

Parameters are laid out in registration order (forward order); backward produces
gradients roughly in reverse, so gradient buckets are formed from the END of the
buffer (``parallel/ddp.py``).
"""
from __future__ import annotations

import math
from typing import Callable, Sequence

import numpy as np
import torch

ALIGN = 64  # elements (256 B fp32): every parameter starts on a 256-B boundary


class Param:
    """Handle of one trainable tensor living in a :class:`ParamArena`."""

    __slots__ = ("name", "shape", "init", "master", "data", "grad", "offset", "trainable", "keras_shape",
                 "to_keras", "from_keras", "_initial")

    def __init__(self, name: str, shape: Sequence[int], init: Callable, trainable: bool = True):
        self.name = name
        self.shape = tuple(int(s) for s in shape)
        self.init = init
        self.master = None
        self.data = None
        self.grad = None
        self.offset = None
        self.trainable = trainable
        self._initial = None
        # Keras-layout conversion (identity by default)
        self.to_keras = lambda a: a
        self.from_keras = lambda a: a

    @property
    def numel(self) -> int:
        return int(math.prod(self.shape))

    def __repr__(self):
        return f"Param({self.name}, {self.shape})"


class ParamArena:
    def __init__(self, params: Sequence[Param], device="cpu", compute_dtype=torch.float32, seed: int | None = 0):
        self.params = list(params)
        self.device = torch.device(device)
        self.compute_dtype = compute_dtype
        off = 0
        for p in self.params:
            p.offset = off
            off += math.ceil(p.numel / ALIGN) * ALIGN
        self.numel = max(off, ALIGN)
        self.master = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        if compute_dtype == torch.float32:
            self.compute = self.master
        else:
            self.compute = torch.zeros(self.numel, dtype=compute_dtype, device=self.device)
        gen = torch.Generator().manual_seed(seed if seed is not None else 0)
        host = torch.zeros(self.numel, dtype=torch.float32)
        for p in self.params:
            if p._initial is not None:
                v = torch.as_tensor(p._initial, dtype=torch.float32).reshape(p.shape)
            else:
                v = p.init(p.shape, gen).to(torch.float32)
            host[p.offset : p.offset + p.numel] = v.reshape(-1)
        self.master.copy_(host)
        for p in self.params:
            sl = slice(p.offset, p.offset + p.numel)
            p.master = self.master[sl].view(p.shape)
            p.grad = self.grad[sl].view(p.shape)
            p.data = self.compute[sl].view(p.shape)
            # Graph anchors: ops take these views and return None for them in backward
            # (their gradients go out of band into ``p.grad``), but marking them makes
            # autograd record every op even when the network input needs no gradient.
            p.data.requires_grad_(True)
            if p.master is not p.data:
                p.master.requires_grad_(True)
        self.sync_compute()

    # -------------------------------------------------------------------------
    def zero_grad(self):
        self.grad.zero_()

    def sync_compute(self):
        from ..ops.optim import cast_master_to_compute

        cast_master_to_compute(self.master, None if self.compute is self.master else self.compute)

    def get_flat(self) -> torch.Tensor:
        return self.master

    def set_flat(self, flat: torch.Tensor):
        self.master.copy_(flat.to(self.master.device, torch.float32))
        self.sync_compute()

    def nbytes(self) -> int:
        n = self.master.numel() * 4 + self.grad.numel() * 4
        if self.compute is not self.master:
            n += self.compute.numel() * self.compute.element_size()
        return n


# ----------------------------------------------------------------------------- initialisers
def zeros(shape, gen):
    return torch.zeros(shape)


def ones(shape, gen):
    return torch.ones(shape)


def constant(v):
    return lambda shape, gen: torch.full(shape, float(v))


def uniform(a):
    return lambda shape, gen: (torch.rand(shape, generator=gen) * 2 - 1) * a


def normal(std):
    return lambda shape, gen: torch.randn(shape, generator=gen) * std


def glorot_uniform(fan_in: int, fan_out: int):
    lim = math.sqrt(6.0 / (fan_in + fan_out))
    return uniform(lim)


def he_normal(fan_in: int):
    return normal(math.sqrt(2.0 / fan_in))


def truncated_normal(std):
    def f(shape, gen):
        t = torch.randn(shape, generator=gen) * std
        return t.clamp_(-2 * std, 2 * std)
    return f


def orthogonal(rows: int, cols: int, gain: float = 1.0):
    """Keras orthogonal initializer for a [rows, cols] matrix (returned in that shape)."""
    def f(shape, gen):
        a = torch.randn((max(rows, cols), min(rows, cols)), generator=gen, dtype=torch.float64)
        q, r = torch.linalg.qr(a)
        q = q * torch.sign(torch.diagonal(r))
        if rows < cols:
            q = q.T
        return (gain * q[:rows, :cols]).to(torch.float32).reshape(shape)
    return f


def to_numpy(t: torch.Tensor) -> np.ndarray:
    return t.detach().to("cpu", torch.float32).numpy().copy()
