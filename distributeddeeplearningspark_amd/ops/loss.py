"""Losses.  ``softmax_cross_entropy`` is ONE fused HIP kernel that returns the loss and
stores dlogits during the forward sweep (the backward only hands them out)."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import zpad as ZP
from ._native import C, use_native


# The root node of a ``loss.backward()`` a training step runs from a unit seed (models/core.py
# backward_unit): that loss node hands out its stored gradient as is — no scaling launch.  Only the
# root qualifies: a loss node inside a user's composite loss receives a non-unit gradient.
_UNIT_SEED = [None]


def unit_seed(ctx) -> bool:
    return ctx is _UNIT_SEED[0]


# small heads (B x K up to 16K logits: MNIST's 16 x 10): one workgroup computes every row AND the batch loss;
# larger ones (ResNet-50's 256 x 1000) keep a workgroup per row + one reduce launch (a single workgroup
# walking 256K logits measured ~0.1 ms/step slower)
_SMALL_LOGITS = 16384


class _SoftmaxXentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, probs, smoothing, ignore_index):
        B, K = logits.shape
        if use_native(logits):
            if logits.stride(1) != 1:
                logits = logits.contiguous()
            ld = logits.stride(0)
            # dlogits in the logits' layout; the kernel zeroes the columns past K, so a padded logits row
            # (ops/zpad.py: a Dense(10) head writes [B, 16]) gives zero-padded dlogits the Dense reads as is
            dfull = torch.empty((B, ld), dtype=logits.dtype, device=logits.device)
            dl = ZP.logical(dfull, K)
            loss = torch.empty(1, dtype=torch.float32, device=logits.device)
            small = B * K <= _SMALL_LOGITS
            rows = None if small else torch.empty(B, dtype=torch.float32, device=logits.device)
            if labels is not None:
                # 1 / #valid labels on the device (no host sync): the gradient scale and the loss normaliser
                inv = torch.empty(1, dtype=torch.float32, device=logits.device)
                lab = labels.to(torch.int64).contiguous()
                C().label_count_inv(lab, ignore_index, inv)
                C().softmax_xent(logits, lab, None, rows, dl, 1.0, smoothing, ignore_index, inv,
                                 loss if small else None, 1.0)
                if not small:
                    C().rows_sum_scaled(rows, 1.0, inv, loss)
            else:
                C().softmax_xent(logits, None, probs.to(torch.float32).contiguous(), rows, dl, 1.0 / B, 0.0, -100,
                                 None, loss if small else None, 1.0 / B)
                if not small:
                    C().rows_sum_scaled(rows, 1.0 / B, None, loss)
            ctx.save_for_backward(dl)
            return loss.view(())
        with torch.enable_grad():
            lg = logits.detach().requires_grad_(True)
            lp = F.log_softmax(lg.float(), dim=-1)
            if labels is not None:
                loss = F.nll_loss(lp, labels.long(), ignore_index=ignore_index, reduction="none")
                if smoothing > 0:
                    sm = -lp.mean(dim=-1)
                    loss = (1 - smoothing) * loss + smoothing * sm * (labels != ignore_index)
                valid = (labels != ignore_index).sum().clamp_min(1)
                out = loss.sum() / valid
            else:
                out = -(probs.float() * lp).sum(-1).mean()
            (dl,) = torch.autograd.grad(out, [lg])
        ctx.save_for_backward(dl)
        return out.detach()

    @staticmethod
    def backward(ctx, g):
        (dl,) = ctx.saved_tensors
        if unit_seed(ctx):
            return dl, None, None, None, None
        return (dl * g.to(dl.dtype)).to(dl.dtype), None, None, None, None


def softmax_cross_entropy(logits, labels=None, probs=None, label_smoothing=0.0, ignore_index=-100):
    """Mean CE of softmax(logits) against class ``labels`` or target ``probs`` rows."""
    if (labels is None) == (probs is None):
        raise ValueError("pass exactly one of labels / probs")
    return _SoftmaxXentFn.apply(logits, labels, probs, float(label_smoothing), int(ignore_index))


class _MSEFn(torch.autograd.Function):
    """One HIP launch computes the loss and stores d loss / d pred (backward = one scale)."""

    @staticmethod
    def forward(ctx, pred, target):
        p = pred.contiguous()
        loss = torch.empty((), dtype=torch.float32, device=p.device)
        grad = torch.empty_like(p)
        C().mse_fwd_bwd(p, target.contiguous(), loss, grad)
        ctx.save_for_backward(grad)
        return loss

    @staticmethod
    def backward(ctx, g):
        (grad,) = ctx.saved_tensors
        return (grad if unit_seed(ctx) else grad * g), None


def mean_squared_error(pred, target):
    if use_native(pred) and pred.dtype == torch.float32 and target.dtype == torch.float32 \
            and pred.shape == target.shape:
        return _MSEFn.apply(pred, target)
    return ((pred.float() - target.float()) ** 2).mean()


def mean_absolute_error(pred, target):
    return (pred.float() - target.float()).abs().mean()


def binary_crossentropy(pred, target, eps=1e-7):
    p = pred.float().clamp(eps, 1 - eps)
    t = target.float()
    return -(t * torch.log(p) + (1 - t) * torch.log(1 - p)).mean()


class _ProbXentFn(torch.autograd.Function):
    """Keras cross-entropy on probabilities (``-sum y log clip(p, eps, 1 - eps)``, batch mean): one HIP
    sweep writes the per-row losses and d loss / d p; a second reduces the rows (no ATen on the GPU)."""

    @staticmethod
    def forward(ctx, probs, labels, target, eps, ignore_index):
        p = probs.float().contiguous()
        B = p.shape[0]
        rows = torch.empty(B, dtype=torch.float32, device=p.device)
        dp = torch.empty_like(p)
        C().prob_xent(p, None if labels is None else labels.to(torch.int64).contiguous(),
                      None if target is None else target.float().contiguous(), rows, dp, float(eps), 1.0 / B,
                      int(ignore_index))
        loss = torch.empty((), dtype=torch.float32, device=p.device)
        C().rows_sum_scaled(rows, 1.0 / B, None, loss.view(1))
        ctx.save_for_backward(dp)
        ctx.in_dtype = probs.dtype
        return loss

    @staticmethod
    def backward(ctx, g):
        (dp,) = ctx.saved_tensors
        if unit_seed(ctx) and dp.dtype == ctx.in_dtype:
            return dp, None, None, None, None
        return (dp * g).to(ctx.in_dtype), None, None, None, None


def prob_cross_entropy(probs, labels=None, target=None, eps=1e-7, ignore_index=-100):
    """Mean Keras CE of probability rows ``probs`` [B, K] against class ``labels`` [B] (sparse form) or
    target rows [B, K] (``categorical_crossentropy`` on a model whose softmax is an output layer)."""
    if (labels is None) == (target is None):
        raise ValueError("pass exactly one of labels / target")
    if use_native(probs):
        return _ProbXentFn.apply(probs, labels, target, eps, ignore_index)
    p = probs.float().clamp(eps, 1 - eps)
    if labels is not None:
        lab = labels.long().reshape(-1)
        keep = (lab != ignore_index) & (lab >= 0) & (lab < p.shape[1])
        picked = torch.log(p.gather(1, lab.clamp(0, p.shape[1] - 1)[:, None])[:, 0])
        return -(picked * keep).sum() / p.shape[0]
    return -(target.float() * torch.log(p)).sum(-1).mean()


def categorical_crossentropy_probs(probs, target, eps=1e-7):
    """Keras semantics on already-softmaxed outputs: -sum(y*log(clip(p)))."""
    return prob_cross_entropy(probs.reshape(probs.shape[0], -1), target=target.reshape(probs.shape[0], -1), eps=eps)
