"""Reference (PyTorch, CPU-first) helpers for the op layer.

Every op of the framework has two implementations: the HIP kernels (GPU) and a
reference built from stock PyTorch ops.  The reference backward is obtained by
re-running the reference forward under autograd, so each op only has to define
its forward math once for the CPU path and for the numerics tests.
"""
from __future__ import annotations

import torch


def ref_grads(fn, inputs, grad_out):
    """Gradients of ``fn(*inputs)`` w.r.t. every floating input (None for the rest)."""
    leaves = []
    for t in inputs:
        if isinstance(t, torch.Tensor) and t.is_floating_point():
            leaves.append(t.detach().requires_grad_(True))
        else:
            leaves.append(t)
    with torch.enable_grad():
        out = fn(*leaves)
        req = [l for l in leaves if isinstance(l, torch.Tensor) and l.requires_grad]
        grads = torch.autograd.grad(out, req, grad_out, allow_unused=True)
    it = iter(grads)
    res = []
    for l in leaves:
        if isinstance(l, torch.Tensor) and l.requires_grad:
            res.append(next(it))
        else:
            res.append(None)
    return res


def accumulate(buf, g):
    """``buf += g`` for an out-of-band gradient buffer (None-safe)."""
    if buf is not None and g is not None:
        buf.add_(g.to(buf.dtype).reshape(buf.shape))
