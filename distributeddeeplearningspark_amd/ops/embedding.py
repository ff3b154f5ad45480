"""Embedding lookup with out-of-band gradient accumulation into the parameter arena."""
from __future__ import annotations

import torch

from ._native import C, use_native


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, w, gw, hook):
        ctx.hook = hook
        ctx.gw = gw
        ctx.save_for_backward(idx)
        ctx.shape = w.shape
        if use_native(w) and hasattr(C(), "embedding_fwd"):
            out = torch.empty((*idx.shape, w.shape[1]), dtype=w.dtype, device=w.device)
            C().embedding_fwd(idx.contiguous().long(), w, out)
            ctx.native = True
            return out
        ctx.native = False
        return torch.nn.functional.embedding(idx.long(), w)

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        gw = ctx.gw
        if gw is not None:
            if ctx.native and hasattr(C(), "embedding_bwd"):
                C().embedding_bwd(idx.contiguous().long(), dy.contiguous(), gw)
            else:
                gw.index_add_(0, idx.reshape(-1).long(), dy.reshape(-1, ctx.shape[1]).to(gw.dtype))
        if ctx.hook is not None:
            ctx.hook()
        return None, None, None, None


def embedding(idx, w, *, grad_w=None, on_grad=None):
    return _EmbeddingFn.apply(idx, w, grad_w, on_grad)
