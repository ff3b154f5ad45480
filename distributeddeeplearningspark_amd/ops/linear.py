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
from . import zpad as ZP
from ._native import C, use_native
from .streams import on_grad_stream
from ._ref import accumulate, ref_grads


def linear_ref(x, w, b, relu=False):
    y = F.linear(x, w, b)
    return torch.relu(y) if relu else y


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, gw, gb, cfg):
        relu, hook, pads = cfg
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
            K, N = x.shape[-1], w.shape[0]
            Kp, Np = ZP.r8(K), ZP.r8(N)
            ctx.pad = (K, N, Kp, Np)
            if pads is not None:
                # padded arena storage (params.py): the GEMMs read / accumulate into it directly
                w, b, gw, gb = pads
            elif Kp != K or Np != N:  # 16-B vector alignment of every GEMM operand row
                w = F.pad(w.detach(), (0, Kp - K, 0, Np - N))
                b = None if b is None else F.pad(b.detach(), (0, Np - N))
                ctx.grad_tmp = True  # logical-shape gradient buffers: padded temporaries in backward
            lead = x.shape[:-1]
            x2 = ZP.padded(x, Kp).view(-1, Kp) if Kp != K else x.reshape(-1, K).contiguous()
            y = torch.empty((*lead, Np), dtype=torch.bfloat16, device=x.device)
            G.linear_fwd(x2, w, bias=b, relu=relu, out=y.view(-1, Np))
            ctx.gw, ctx.gb = gw, gb
            ctx.save_for_backward(x2, w, y.view(-1, Np) if relu else None)
            return ZP.logical(y, N)  # zero-padded storage: the next Dense reads it as is
        y = linear_ref(x, w.to(x.dtype), None if b is None else b.to(x.dtype), relu)
        ctx.gw, ctx.gb = gw, gb
        ctx.save_for_backward(x, w, b)
        return y

    @staticmethod
    def backward(ctx, dy):
        relu, hook, _ = ctx.cfg
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
            lead = ctx.xshape[:-1]
            d2 = (ZP.padded(dy, Np) if Np != N else dy.contiguous()).view(-1, Np)
            if getattr(ctx, "grad_tmp", False):  # logical-shape gradient buffers: padded temporaries
                tgw = None if gw is None else torch.zeros((Np, Kp), dtype=torch.float32, device=d2.device)
                tgb = None if gb is None else torch.zeros(Np, dtype=torch.float32, device=d2.device)
            else:
                tgw, tgb = gw, gb
            with on_grad_stream(d2.device, d2, x2, default=False):  # parameter gradients beside the data-gradient
                if relu:
                    t = torch.empty_like(d2)
                    if tgb is not None:  # ReLU backward fused into the bias-gradient sweep
                        C().bias_grad(d2, tgb, Np, True, y, t)
                    else:
                        C().relu_bwd(d2, y, t)
                    d2 = t
                elif tgb is not None:
                    C().bias_grad(d2, tgb, Np, True)
                if tgw is not None:
                    G.linear_wgrad(d2, x2, tgw)
            if tgw is not gw and gw is not None:
                gw.add_(tgw[:N, :K])
            if tgb is not gb and gb is not None:
                gb.add_(tgb[:N])
            if ctx.needs_dx:
                dxp = torch.empty((*lead, Kp), dtype=torch.bfloat16, device=d2.device)
                G.linear_dgrad(d2, w, out=dxp.view(-1, Kp))
                dx = ZP.logical(dxp, K)  # zero columns past K (the padded weight columns are zero)
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


def linear(x, w, bias=None, *, relu=False, grad_w=None, grad_b=None, on_grad=None, padded=None):
    """``padded``: (weight, bias, weight grad, bias grad) zero-padded arena storage ([Np, Kp], [Np], N and K
    rounded up to multiples of 8; ``models/params.py``) used by the GPU GEMMs in place of the logical
    ``w`` / ``bias`` / ``grad_w`` / ``grad_b``."""
    return _LinearFn.apply(x, w, bias, grad_w, grad_b, (bool(relu), on_grad, padded))
