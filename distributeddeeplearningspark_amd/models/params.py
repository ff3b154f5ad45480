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

Padded storage: a layer may ask for a parameter's storage to be wider than its shape
(``Param(pad=...)``, e.g. a Dense(225) kernel [225, 4608] kept as [232, 4608], a
Conv2D(1 -> 32) filter [32, 3, 3, 1] as [32, 3, 3, 8]) so the MFMA GEMMs, whose operand rows are
read as 16-B vectors, use the arena storage directly instead of padded copies made every step.
Bf16 arenas honour the request (fp32 arenas: the fp32 GEMM takes element strides); the padding
is zero in the master, compute and gradient buffers and stays zero (its gradients are zero, so
every optimizer leaves it at zero).  ``p.master / p.data / p.grad`` are the logical views (the
Keras surface); ``p.pmaster / p.pdata / p.pgrad`` the padded storage views.

Flat weights that leave the arena (``get_flat`` / ``set_flat``: serialised models, worker results,
checkpoints, parameter-server traffic) use the CANONICAL layout — the unpadded one an fp32 arena has —
so a bf16 GPU worker, the fp32 CPU driver and a checkpoint all agree; ``master`` / ``grad`` and the
device-side exchanges between workers of one layout stay in the storage layout.
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
                 "to_keras", "from_keras", "_initial", "pad", "pshape", "pmaster", "pdata", "pgrad")

    def __init__(self, name: str, shape: Sequence[int], init: Callable, trainable: bool = True, pad=None):
        self.name = name
        self.shape = tuple(int(s) for s in shape)
        # requested storage shape (>= shape per dim); pshape: the one the arena chose
        self.pad = None if pad is None else tuple(max(int(a), int(b)) for a, b in zip(pad, self.shape))
        self.pshape = self.shape
        self.pmaster = self.pdata = self.pgrad = None
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

    @property
    def snumel(self) -> int:
        """Elements of the arena storage (the padded shape)."""
        return int(math.prod(self.pshape))

    @property
    def padded(self) -> bool:
        return self.pshape != self.shape

    @property
    def logical(self) -> tuple:
        """Index of the logical region inside the padded storage."""
        return tuple(slice(0, n) for n in self.shape)

    def __repr__(self):
        return f"Param({self.name}, {self.shape})"


class ParamArena:
    def __init__(self, params: Sequence[Param], device="cpu", compute_dtype=torch.float32, seed: int | None = 0):
        self.params = list(params)
        self.device = torch.device(device)
        self.compute_dtype = compute_dtype
        off = 0
        for p in self.params:
            p.pshape = p.pad if (p.pad is not None and compute_dtype != torch.float32) else p.shape
            p.offset = off
            off += math.ceil(p.snumel / ALIGN) * ALIGN
        self.numel = max(off, ALIGN)
        self.padded = any(p.padded for p in self.params)
        # canonical (unpadded) layout: offsets of an fp32 arena over the same parameters
        self.canon_offsets, coff = [], 0
        for p in self.params:
            self.canon_offsets.append(coff)
            coff += math.ceil(p.numel / ALIGN) * ALIGN
        self.canon_numel = max(coff, ALIGN)
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
            if p.padded:
                host[p.offset : p.offset + p.snumel].view(p.pshape)[p.logical] = v
            else:
                host[p.offset : p.offset + p.numel] = v.reshape(-1)
        self.master.copy_(host)
        self._bind_views()
        self.sync_compute()

    def _bind_views(self):
        for p in self.params:
            sl = slice(p.offset, p.offset + p.snumel)
            p.pmaster = self.master[sl].view(p.pshape)
            p.pgrad = self.grad[sl].view(p.pshape)
            p.pdata = self.compute[sl].view(p.pshape)
            if p.padded:
                p.master, p.grad, p.data = p.pmaster[p.logical], p.pgrad[p.logical], p.pdata[p.logical]
            else:
                p.master, p.grad, p.data = p.pmaster, p.pgrad, p.pdata
            # Graph anchors: ops take these views and return None for them in backward
            # (their gradients go out of band into ``p.grad``), but marking them makes
            # autograd record every op even when the network input needs no gradient.
            p.data.requires_grad_(True)
            if p.master is not p.data:
                p.master.requires_grad_(True)

    def rebind(self, master: torch.Tensor, grad: torch.Tensor, compute: torch.Tensor):
        """Move the arena into caller-provided flat buffers (same layout; their current contents are kept):
        a replica group stacks its replicas' arenas in one [R, numel] allocation so that one launch can
        address every replica's weights at a fixed stride (parallel/replica_seq.py).  Layers read the new
        views from their Params at the next call."""
        assert master.numel() == grad.numel() == compute.numel() == self.numel
        self.master, self.grad = master, grad
        self.compute = master if self.compute_dtype == torch.float32 else compute
        self._bind_views()

    # -------------------------------------------------------------------------
    grads_zeroed = False  # set by a captured optimizer update that zeroed the gradients it consumed

    def zero_grad(self, defer: bool = False):
        """Zero the gradient arena; ``defer``: return the arena for the caller to zero (with the step's
        other workspaces in one launch, ``ops.norm.reset_workspaces``) instead."""
        if self.grads_zeroed:  # the previous (captured) update left them zero: no fill launch
            self.grads_zeroed = False
            return None
        if defer:
            return self.grad
        self.grad.zero_()
        return None

    def sync_compute(self):
        from ..ops.optim import cast_master_to_compute

        cast_master_to_compute(self.master, None if self.compute is self.master else self.compute)

    def to_canonical(self, t: torch.Tensor) -> torch.Tensor:
        """A storage-layout flat (``master``, a worker's final weights, a delta) in the canonical layout."""
        if not self.padded:
            return t
        out = t.new_zeros(self.canon_numel)
        for p, co in zip(self.params, self.canon_offsets):
            out[co:co + p.numel].view(p.shape).copy_(t[p.offset:p.offset + p.snumel].view(p.pshape)[p.logical])
        return out

    def from_canonical(self, c: torch.Tensor) -> torch.Tensor:
        """A canonical flat in the storage layout (zero padding)."""
        if not self.padded:
            return c
        out = c.new_zeros(self.numel)
        for p, co in zip(self.params, self.canon_offsets):
            out[p.offset:p.offset + p.snumel].view(p.pshape)[p.logical].copy_(c[co:co + p.numel].view(p.shape))
        return out

    def get_flat(self) -> torch.Tensor:
        """The fp32 weights as a canonical flat (``master`` itself when nothing is padded)."""
        return self.to_canonical(self.master)

    def set_flat(self, flat: torch.Tensor):
        """Load a canonical flat (``get_flat`` of any arena over the same parameters)."""
        if flat.numel() != self.canon_numel:
            raise ValueError(f"set_flat: {flat.numel()} elements, the canonical layout has {self.canon_numel}")
        with torch.no_grad():
            self.master.copy_(self.from_canonical(flat.to(self.master.device, torch.float32)))
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
