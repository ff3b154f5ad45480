"""Zero-padded activations: the 16-B row granularity of the MFMA GEMM operands, kept across layers.

A GEMM operand row is read as 16-B vectors (8 bf16), so a Dense(225) output or a 1-channel image has
to be padded to 232 / 8 columns before a GEMM reads it.  Weights are padded once, in the arena
(``models/params.py``); activations are padded by their PRODUCER: a layer whose output width is not a
multiple of 8 allocates ``[..., Np]`` storage whose extra columns are zero, marks that storage, and
returns the logical ``[..., N]`` view of it.  A consumer that wants the padded operand reads the view's
base (``base``), so a Dense(225) -> Dense(10) -> softmax-xent chain runs with no pad / slice copies in
either direction — the reference's MNIST head (``ddl_mnist_aztk.py:186-190``) is exactly that chain.
Gradients travel the same way (the loss writes zero-padded dlogits, a Dense dgrad zero columns).

Only tensors allocated by this package's ops carry the mark, so a user's strided view of some
other buffer is never mistaken for zero-padded storage.
"""
from __future__ import annotations

import torch

from ._native import C


def r8(n: int) -> int:
    return -(-int(n) // 8) * 8


def mark(t: torch.Tensor) -> torch.Tensor:
    """Declare ``t`` zero-padded storage (its columns past the consumer's logical width are zero)."""
    t._ddl_zpad = True
    return t


def logical(storage: torch.Tensor, n: int) -> torch.Tensor:
    """The ``[..., n]`` view of marked padded storage (``storage`` itself when it is not wider)."""
    if storage.shape[-1] == n:
        return storage
    return mark(storage)[..., :n]


def base(t: torch.Tensor, width: int):
    """The marked ``[..., width]`` zero-padded storage ``t`` is the leading-column view of, else None."""
    if t.shape[-1] == width and t.is_contiguous():
        return t
    b = t._base
    if b is None or not getattr(b, "_ddl_zpad", False) or b.shape[-1] != width or b.dim() != t.dim():
        return None
    if b.shape[:-1] != t.shape[:-1] or t.data_ptr() != b.data_ptr() or t.stride() != b.stride():
        return None
    return b


def padded(t: torch.Tensor, width: int) -> torch.Tensor:
    """``t`` [..., K] as contiguous zero-padded ``[..., width]`` storage: its marked base when it has
    one, else a padded copy (one HIP pass)."""
    b = base(t, width)
    if b is not None:
        return b
    out = torch.empty((*t.shape[:-1], width), dtype=t.dtype, device=t.device)
    if t.stride(-1) != 1 or any(t.stride(d) != t.stride(d + 1) * t.shape[d + 1] for d in range(t.dim() - 2)):
        t = t.contiguous()
    C().pad_cols_bf16(t, out)
    return mark(out)
