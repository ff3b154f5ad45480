"""Keras-2 recurrent cells (GRU ``reset_after=False``, LSTM, SimpleRNN).

Math (Keras 2, the reference's GRU/LSTM, ``ddl_nyiso_aztk.py:201-203,249-251``):
  GRU : z = hs(x Wz + h Uz + bz); r = hs(x Wr + h Ur + br);
        hh = tanh(x Wh + (r*h) Uh + bh); h = z*h + (1-z)*hh
  LSTM: i,f,o = hs(x W + h U + b) (gate order i,f,c,o); c = f*c + i*tanh(...); h = o*tanh(c)
with hs = hard_sigmoid = clip(0.2x+0.5, 0, 1).

The whole input projection x@W for all T steps is ONE fp32 MFMA GEMM (or fused into the
register-resident kernel for narrow inputs); the recurrence runs in the persistent HIP kernels
(``csrc/kernels/rnn.hip``): the register-resident fast path for the Keras defaults (tanh +
hard_sigmoid, H = 64/128), the generic kernels for every other activation pair, SimpleRNN and
other widths.  CPU tensors use the reference path below.  Parameter gradients accumulate
into the arena in one launch.
"""
from __future__ import annotations

import torch

from ._native import C, use_native
from ._ref import accumulate, ref_grads


def _act(name):
    from .act import activation_ref

    if name == "softmax" or name == "gelu":
        raise ValueError(f"unsupported recurrent activation {name!r}")
    return lambda x: activation_ref(name, x)


def recurrent_ref(cell, x, W, U, b, return_sequences, activation="tanh", recurrent_activation="hard_sigmoid"):
    B, T, _ = x.shape
    H = U.shape[0]
    act, ract = _act(activation), _act(recurrent_activation)
    xw = x @ W
    if b is not None:
        xw = xw + b
    h = x.new_zeros((B, H))
    c = x.new_zeros((B, H))
    outs = []
    for t in range(T):
        xt = xw[:, t]
        if cell == "gru":
            hu = h @ U[:, : 2 * H]
            z = ract(xt[:, :H] + hu[:, :H])
            r = ract(xt[:, H : 2 * H] + hu[:, H:])
            hh = act(xt[:, 2 * H :] + (r * h) @ U[:, 2 * H :])
            h = z * h + (1 - z) * hh
        elif cell == "lstm":
            g = xt + h @ U
            i = ract(g[:, :H])
            f = ract(g[:, H : 2 * H])
            cc = act(g[:, 2 * H : 3 * H])
            o = ract(g[:, 3 * H :])
            c = f * c + i * cc
            h = o * act(c)
        else:
            h = act(xt + h @ U)
        if return_sequences:
            outs.append(h)
    return torch.stack(outs, 1) if return_sequences else h


class _RecurrentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, U, b, gW, gU, gb, cfg):
        cell, rs, act, ract, hook = cfg
        ctx.cfg = cfg
        dt = x.dtype
        xf, Wf, Uf = x.float(), W.float(), U.float()
        bf = None if b is None else b.float()
        if use_native(x):
            codes = C().ACT_CODES
            for a in (act, ract):
                if a not in codes or a == "gelu":
                    raise ValueError(f"recurrent activation {a!r} has no HIP kernel (supported: "
                                     f"{sorted(k for k in codes if k != 'gelu')})")
            ctx.codes = (codes[act], codes[ract])
            y, saved = C().rnn_fwd(cell, xf.contiguous(), Wf.contiguous(), Uf.contiguous(), bf, rs, *ctx.codes)
            ctx.native = True
            ctx.grads = (gW, gU, gb)
            ctx.needs_dx = ctx.needs_input_grad[0]
            ctx.save_for_backward(xf, Wf, Uf, bf, *saved)
            return y.to(dt)
        ctx.native = False
        with torch.no_grad():
            y = recurrent_ref(cell, xf, Wf, Uf, bf, rs, act, ract)
        ctx.grads = (gW, gU, gb)
        ctx.save_for_backward(xf, Wf, Uf, bf)
        return y.to(dt)

    @staticmethod
    def backward(ctx, dy):
        cell, rs, act, ract, hook = ctx.cfg
        saved = ctx.saved_tensors
        xf, Wf, Uf, bf = saved[:4]
        gW, gU, gb = ctx.grads
        if ctx.native:
            # fast path: dW/dU/db are accumulated into the fp32 arena slices in-kernel (None here)
            fp32 = lambda t: t if t is not None and t.dtype == torch.float32 and t.is_contiguous() else None
            dx, dW, dU, db = C().rnn_bwd(cell, dy.float().contiguous(), xf, Wf, Uf, bf, rs, list(saved[4:]),
                                         fp32(gW), fp32(gU), fp32(gb), ctx.needs_dx, *ctx.codes)
        else:
            fn = lambda xx, ww, uu, bb: recurrent_ref(cell, xx, ww, uu, bb, rs, act, ract)
            dx, dW, dU, db = ref_grads(fn, [xf, Wf, Uf, bf], dy.float())
        accumulate(gW, dW)
        accumulate(gU, dU)
        accumulate(gb, db)
        if hook is not None:
            hook()
        return (None if dx is None else dx.to(dy.dtype)), None, None, None, None, None, None, None


def recurrent(cell, x, W, U, b=None, *, grads=(None, None, None), return_sequences=False, activation="tanh",
              recurrent_activation="hard_sigmoid", on_grad=None):
    gW, gU, gb = grads
    cfg = (cell, bool(return_sequences), activation, recurrent_activation, on_grad)
    return _RecurrentFn.apply(x, W, U, b, gW, gU, gb, cfg)
