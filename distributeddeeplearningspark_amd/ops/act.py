"""Standalone activations, softmax, dropout and average pooling of the Keras layer set.

The flagship models fuse these into GEMM / BatchNorm epilogues; the layers below run when a
user model places them on their own (``Activation('tanh')``, ``Dropout(0.5)``,
``AveragePooling2D``, a ``Dense(..., activation='sigmoid')`` head).  On a GPU every one is a
HIP kernel (``csrc/kernels/layer_ops.hip``); CPU tensors use the PyTorch reference.

Reference usage: ``Activation('relu')`` / ``Activation('softmax')`` in the MNIST CNN
(``ddl_mnist_aztk.py:180-192``).
"""
from __future__ import annotations

import itertools

import torch
import torch.nn.functional as F

from ._native import C, use_native

ACT_NAMES = ("linear", "relu", "tanh", "sigmoid", "hard_sigmoid", "elu", "selu", "softplus", "gelu")


def _code(name: str) -> int:
    return C().ACT_CODES[name]


def activation_ref(name: str, x):
    if name in (None, "linear"):
        return x
    if name == "relu":
        return torch.relu(x)
    if name == "tanh":
        return torch.tanh(x)
    if name == "sigmoid":
        return torch.sigmoid(x)
    if name == "hard_sigmoid":
        return torch.clamp(0.2 * x + 0.5, 0.0, 1.0)
    if name == "elu":
        return F.elu(x)
    if name == "selu":
        return F.selu(x)
    if name == "softplus":
        return F.softplus(x)
    if name == "gelu":
        return F.gelu(x)
    if name == "softmax":
        return torch.softmax(x.float(), dim=-1).to(x.dtype)
    raise ValueError(f"unknown activation {name!r}")


class _ActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, name):
        x = x.contiguous()
        y = torch.empty_like(x)
        code = _code(name)
        C().act_fwd(x, y, code)
        ctx.code = code
        ctx.save_for_backward(x if name == "gelu" else y)  # derivative from y (GELU: from x)
        return y

    @staticmethod
    def backward(ctx, dy):
        (ref,) = ctx.saved_tensors
        dx = torch.empty_like(ref)
        C().act_bwd(dy.contiguous(), ref, dx, ctx.code)
        return dx, None


class _SoftmaxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        y = torch.empty_like(x)
        C().softmax_fwd(x, y)
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dx = torch.empty_like(y)
        C().softmax_bwd(dy.contiguous(), y, dx)
        return dx


def _native_float(x) -> bool:
    return use_native(x) and x.dtype in (torch.float32, torch.bfloat16)


def activation(x, name: str):
    """``name`` in :data:`ACT_NAMES` or ``'softmax'`` (over the last axis)."""
    if name in (None, "linear"):
        return x
    if not _native_float(x):
        return activation_ref(name, x)
    if name == "softmax":
        return _SoftmaxFn.apply(x)
    if name not in ACT_NAMES:
        raise ValueError(f"activation {name!r} has no HIP kernel (supported: {ACT_NAMES + ('softmax',)})")
    return _ActFn.apply(x, name)


# ------------------------------------------------------------------------------------ dropout
_SEEDS = itertools.count(0x5EED)


def _process_rank() -> int:
    """This replica's rank (torch.distributed, else RANK / DDL_WORKER_RANK), 0 when alone."""
    import os

    try:
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized():
            return dist.get_rank()
    except Exception:
        pass
    return int(os.environ.get("RANK", os.environ.get("DDL_WORKER_RANK", "0")) or 0)


def next_seed(base: int | None = None) -> int:
    """A fresh 63-bit dropout seed (host counter): each call draws an independent mask.  The
    default ``base`` is the process rank, so data-parallel replicas draw different masks."""
    b = _process_rank() + 1 if base is None else int(base)
    return (b * 0x9E3779B97F4A7C15 + next(_SEEDS) * 0xBF58476D1CE4E5B9) & 0x7FFFFFFFFFFFFFFF


_DSTEP: dict = {}  # device -> fp32 [1] dropout step counter of graph-replayed steps (models/step.py)


def dropout_step_counter(device) -> torch.Tensor:
    """The device's dropout step counter: a captured step's dropout kernels mix it into their (capture-time) seeds
    and the replayed graph ticks it once per step (``tick_dropout_step``), so every replay draws fresh masks."""
    d = torch.device(device)
    key = (d.type, d.index if d.index is not None else torch.cuda.current_device())
    t = _DSTEP.get(key)
    if t is None:
        t = _DSTEP[key] = torch.zeros(1, dtype=torch.float32, device=d)
    return t


def tick_dropout_step(device):
    """+1 on the device's dropout step counter (one HIP launch; captured at the end of a graph-replayed step)."""
    C().step_tick(dropout_step_counter(device))


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, seed):
        x = x.contiguous()
        y = torch.empty_like(x)
        # inside a hipGraph capture the seed is fixed at capture time: the device counter varies it per replay
        ds = dropout_step_counter(x.device) if torch.cuda.is_current_stream_capturing() else None
        C().dropout(x, y, p, seed, ds)
        ctx.p, ctx.seed, ctx.ds = p, seed, ds
        return y

    @staticmethod
    def backward(ctx, dy):
        dx = torch.empty_like(dy, memory_format=torch.contiguous_format)
        C().dropout(dy.contiguous(), dx, ctx.p, ctx.seed, ctx.ds)  # same counter hash -> same mask
        return dx, None, None


def dropout(x, p: float, training: bool, seed: int | None = None):
    """Inverted dropout (kept elements scaled by 1/(1-p)); identity in inference."""
    if not training or p <= 0.0:
        return x
    if not _native_float(x):
        return F.dropout(x, p, training=True)
    return _DropoutFn.apply(x, float(p), next_seed() if seed is None else int(seed))


# ------------------------------------------------------------------------------ avg pooling
def _out(n, k, s, p):
    return (n + 2 * p - k) // s + 1


def avgpool_ref(x, k, s, p):
    """NHWC average pooling with the padding excluded from the divisor (Keras 'same')."""
    y = F.avg_pool2d(x.permute(0, 3, 1, 2), k, s, p, count_include_pad=False)
    return y.permute(0, 2, 3, 1).contiguous()


class _AvgPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        x = x.contiguous()
        N, H, W, Cc = x.shape
        Ho, Wo = _out(H, k[0], s[0], p[0]), _out(W, k[1], s[1], p[1])
        y = torch.empty((N, Ho, Wo, Cc), dtype=x.dtype, device=x.device)
        C().avgpool2d_fwd(x, y, k[0], k[1], s[0], s[1], p[0], p[1])
        ctx.k, ctx.s, ctx.p, ctx.xshape = k, s, p, x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        dx = torch.empty(ctx.xshape, dtype=dy.dtype, device=dy.device)
        k, s, p = ctx.k, ctx.s, ctx.p
        C().avgpool2d_bwd(dy.contiguous(), dx, k[0], k[1], s[0], s[1], p[0], p[1])
        return dx, None, None, None


def avg_pool2d(x, kernel_size, stride, padding):
    k, s, p = tuple(kernel_size), tuple(stride), tuple(padding)
    if not _native_float(x):
        return avgpool_ref(x, k, s, p)
    return _AvgPoolFn.apply(x, k, s, p)
