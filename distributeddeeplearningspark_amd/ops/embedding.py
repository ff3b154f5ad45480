"""Keras ``Embedding`` lookup with out-of-band gradient accumulation into the parameter arena.

GPU: a row-gather HIP kernel forward and an fp32 scatter-add backward
(``csrc/kernels/layer_ops.hip: embedding_gather / embedding_scatter``) for bf16 or fp32
tables.  Out-of-range ids produce zero rows and set a device flag; ``DDL_CHECK_IDS=1``
makes every eager forward check the flag and raise (one host sync per call).
BERT's fused word+position+type embedding is a separate kernel (``ops/transformer.py``).
"""
from __future__ import annotations

import os

import torch

from ._native import C, use_native


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, w, gw, hook):
        ctx.hook = hook
        ctx.gw = gw
        ctx.shape = w.shape
        ctx.native = use_native(w)
        ids = idx.contiguous().long()
        ctx.save_for_backward(ids)
        if ctx.native:
            out = torch.empty((*idx.shape, w.shape[1]), dtype=w.dtype, device=w.device)
            bad = torch.zeros(1, dtype=torch.int32, device=w.device)
            C().embedding_fwd(ids, w.contiguous(), out, bad)
            if os.environ.get("DDL_CHECK_IDS") == "1" and not torch.cuda.is_current_stream_capturing():
                if int(bad.item()):
                    raise IndexError(f"Embedding: an id is outside [0, {w.shape[0]})")
            return out
        return torch.nn.functional.embedding(ids, w)

    @staticmethod
    def backward(ctx, dy):
        (ids,) = ctx.saved_tensors
        gw = ctx.gw
        if gw is not None:
            if ctx.native:
                C().embedding_bwd(ids, dy.contiguous(), gw)
            else:
                gw.index_add_(0, ids.reshape(-1), dy.reshape(-1, ctx.shape[1]).to(gw.dtype))
        if ctx.hook is not None:
            ctx.hook()
        return None, None, None, None


def embedding(idx, w, *, grad_w=None, on_grad=None):
    return _EmbeddingFn.apply(idx, w, grad_w, on_grad)
