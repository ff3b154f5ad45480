"""Dense layer ``y = act(x @ W^T + b)`` on the MFMA GEMM (bias/ReLU fused in the epilogue).

Weights are stored ``[out, in]`` (K-contiguous for the forward); the data gradient
reads W row-contiguous (``ds_read_b64_tr_b16``) and the weight gradient accumulates
fp32 into the gradient arena.  fp32 models (the reference's Keras regressors) run the same
three contractions on the fp32 MFMA GEMM (``csrc/kernels/gemm_f32.hip``: exact fp32,
element strides instead of transposed copies) with the bias / ReLU in its epilogue.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import gemm as G
from ._native import C, use_native
from .streams import on_grad_stream
from ._ref import accumulate, ref_grads


def linear_ref(x, w, b, relu=False):
    y = F.linear(x, w, b)
    return torch.relu(y) if relu else y


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, gw, gb, cfg):
        relu, hook = cfg
        ctx.cfg = cfg
        ctx.native = use_native(x)
        ctx.xshape = x.shape
        ctx.needs_dx = ctx.needs_input_grad[0]
        ctx.fp32 = ctx.native and x.dtype == torch.float32
        if ctx.fp32:  # fp32 models (the reference's Keras regressors): the fp32 MFMA GEMM
            x2 = x.reshape(-1, x.shape[-1]).contiguous()
            w = w.contiguous()
            M, K, N = x2.shape[0], x2.shape[1], w.shape[0]
            y = torch.empty((M, N), dtype=torch.float32, device=x.device)
            C().gemm_f32(x2, K, 1, w, 1, K, y, N, M, N, K, 1.0, 0.0,
                         None if b is None else b.float().contiguous(), bool(relu))
            ctx.gw, ctx.gb = gw, gb
            ctx.save_for_backward(x2, w, y if relu else None)
            return y.view(*x.shape[:-1], w.shape[0])
        if ctx.native:
            x2 = x.reshape(-1, x.shape[-1]).contiguous()
            K, N = x2.shape[1], w.shape[0]
            Kp, Np = -(-K // 8) * 8, -(-N // 8) * 8
            ctx.pad = (K, N, Kp, Np)
            if Kp != K or Np != N:  # 16-B vector alignment of every GEMM operand row
                x2 = F.pad(x2, (0, Kp - K))
                w = F.pad(w.detach(), (0, Kp - K, 0, Np - N))
                b = None if b is None else F.pad(b.detach(), (0, Np - N))
            y = G.linear_fwd(x2, w, bias=b, relu=relu)
            ctx.gw, ctx.gb = gw, gb
            ctx.save_for_backward(x2, w, y if relu else None)
            if Np != N:
                y = y[:, :N].contiguous()
            return y.view(*x.shape[:-1], N)
        y = linear_ref(x, w.to(x.dtype), None if b is None else b.to(x.dtype), relu)
        ctx.gw, ctx.gb = gw, gb
        ctx.save_for_backward(x, w, b)
        return y

    @staticmethod
    def backward(ctx, dy):
        relu, hook = ctx.cfg
        dx = None
        if ctx.fp32:
            x2, w, y = ctx.saved_tensors
            M, K, N = x2.shape[0], x2.shape[1], w.shape[0]
            d2 = dy.reshape(-1, N).float().contiguous()
            if relu:
                t = torch.empty_like(d2)
                C().act_bwd(d2, y, t, C().ACT_CODES["relu"])
                d2 = t
            if ctx.gb is not None:
                C().colsum_f32(d2, ctx.gb)
            if ctx.gw is not None:  # gw[n][k] += sum_m d2[m][n] x2[m][k]
                C().gemm_f32(d2, 1, N, x2, K, 1, ctx.gw, K, N, K, M, 1.0, 1.0, None, False)
            if ctx.needs_dx:  # dx[m][k] = sum_n d2[m][n] w[n][k]
                dxt = torch.empty((M, K), dtype=torch.float32, device=d2.device)
                C().gemm_f32(d2, N, 1, w, K, 1, dxt, K, M, K, N, 1.0, 0.0, None, False)
                dx = dxt.view(ctx.xshape)
        elif ctx.native:
            x2, w, y = ctx.saved_tensors
            gw, gb = ctx.gw, ctx.gb
            K, N, Kp, Np = ctx.pad
            d2 = dy.reshape(-1, N).contiguous()
            if Np != N:
                d2 = F.pad(d2, (0, Np - N))
            if relu:
                t = torch.empty_like(d2)
                C().relu_bwd(d2, y, t)
                d2 = t
            with on_grad_stream(d2.device, d2, x2, default=False):  # parameter gradients beside the data-gradient
                if gb is not None:
                    C().bias_grad(d2, gb, N, True) if Np == N else gb.add_(d2[:, :N].float().sum(0))
                if gw is not None:
                    if Np == N and Kp == K:
                        G.linear_wgrad(d2, x2, gw)
                    else:
                        tmp = torch.zeros((Np, Kp), dtype=torch.float32, device=d2.device)
                        G.linear_wgrad(d2, x2, tmp)
                        gw.add_(tmp[:N, :K])
            if ctx.needs_dx:
                dxp = G.linear_dgrad(d2, w)
                dx = (dxp[:, :K].contiguous() if Kp != K else dxp).view(ctx.xshape)
        else:
            x, w, b = ctx.saved_tensors
            gw, gb = ctx.gw, ctx.gb
            fn = lambda xx, ww, bb: linear_ref(xx, ww, bb, relu)
            gx, gww, gbb = ref_grads(fn, [x, w.to(x.dtype), None if b is None else b.to(x.dtype)], dy)
            accumulate(gw, gww)
            accumulate(gb, gbb)
            dx = gx if ctx.needs_dx else None
        if hook is not None:
            hook()
        return dx, None, None, None, None, None


def linear(x, w, bias=None, *, relu=False, grad_w=None, grad_b=None, on_grad=None):
    return _LinearFn.apply(x, w, bias, grad_w, grad_b, (bool(relu), on_grad))
