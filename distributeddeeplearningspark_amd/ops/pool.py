"""NHWC max-pooling (byte argmax, gather backward) and global average pooling."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ._native import C, use_native
from ._ref import ref_grads


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


def _out(n, k, s, p):
    return (n + 2 * p - k) // s + 1


def maxpool_ref(x, k, s, p):
    return F.max_pool2d(x.permute(0, 3, 1, 2), k, s, p).permute(0, 2, 3, 1).contiguous()


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        ctx.k, ctx.s, ctx.p = k, s, p
        ctx.native = use_native(x)
        if ctx.native:
            x = x.contiguous()
            N, H, W, Cc = x.shape
            Ho, Wo = _out(H, k[0], s[0], p[0]), _out(W, k[1], s[1], p[1])
            y = torch.empty((N, Ho, Wo, Cc), dtype=x.dtype, device=x.device)
            am = torch.empty((N, Ho, Wo, Cc), dtype=torch.uint8, device=x.device)
            C().maxpool_fwd(x, y, am, k[0], k[1], s[0], s[1], p[0], p[1])
            ctx.save_for_backward(am)
            ctx.xshape = x.shape
            return y
        ctx.save_for_backward(x)
        return maxpool_ref(x, k, s, p)

    @staticmethod
    def backward(ctx, dy):
        k, s, p = ctx.k, ctx.s, ctx.p
        if ctx.native:
            (am,) = ctx.saved_tensors
            dx = torch.empty(ctx.xshape, dtype=dy.dtype, device=dy.device)
            C().maxpool_bwd(dy.contiguous(), am, dx, k[0], k[1], s[0], s[1], p[0], p[1])
            return dx, None, None, None
        (x,) = ctx.saved_tensors
        (dx,) = ref_grads(lambda xx: maxpool_ref(xx, k, s, p), [x], dy)
        return dx, None, None, None


def max_pool2d(x, kernel_size, stride=None, padding=0):
    k = _pair(kernel_size)
    s = _pair(stride if stride is not None else kernel_size)
    return _MaxPoolFn.apply(x, k, s, _pair(padding))


class _GlobalAvgPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.native = use_native(x)
        ctx.xshape = x.shape
        if ctx.native:
            x = x.contiguous()
            y = torch.empty((x.shape[0], x.shape[-1]), dtype=x.dtype, device=x.device)
            C().avgpool_fwd(x, y)
            return y
        return x.mean(dim=(1, 2))

    @staticmethod
    def backward(ctx, dy):
        if ctx.native:
            dx = torch.empty(ctx.xshape, dtype=dy.dtype, device=dy.device)
            C().avgpool_bwd(dy.contiguous(), dx)
            return dx
        N, H, W, Cc = ctx.xshape
        return (dy / (H * W)).view(N, 1, 1, Cc).expand(N, H, W, Cc).contiguous()


def global_avg_pool(x):
    """[N, H, W, C] -> [N, C]."""
    return _GlobalAvgPoolFn.apply(x)
