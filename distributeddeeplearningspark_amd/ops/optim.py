"""Flat-buffer optimizer steps (one launch per step for the whole model).

GPU: ``csrc/kernels/optim.hip`` (fp32 master update + bf16 compute-copy write in the
same sweep).  CPU: the identical math with vectorised torch ops on the flat tensors.
"""
from __future__ import annotations

import torch

from ._native import C, use_native


def sgd_(w, g, mom, w16, *, lr, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False, grad_scale=1.0):
    if use_native(w):
        C().sgd_step(w, g, mom, w16, lr, momentum, dampening, weight_decay, nesterov, grad_scale)
        return
    d = g * grad_scale
    if weight_decay:
        d = d + weight_decay * w
    if momentum:
        mom.mul_(momentum).add_(d, alpha=1.0 - dampening)
        d = d + momentum * mom if nesterov else mom
    w.sub_(lr * d)
    if w16 is not None and w16.data_ptr() != w.data_ptr():
        w16.copy_(w)


def adam_(w, g, m, v, w16, *, lr, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0, decoupled=False,
          keras_eps=False, step=1, grad_scale=1.0, device_step=None, tick_ctr=None, zero_grad=False):
    """``device_step``: optional fp32 GPU scalar holding the step count, already advanced for
    this step by :func:`step_tick` (the optimizer does it once per step, before the first
    ranged update); the bias corrections are computed from it on the device (graph-replay safe).
    ``tick_ctr`` (int32 [1], zeroed once): the launch advances ``device_step`` itself (no step_tick
    launch); ``zero_grad``: ``g`` is zeroed as it is consumed.  Both GPU only (captured steps)."""
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    if use_native(w):
        mode = (1 if decoupled else 0) | (2 if keras_eps else 0) | (4 if tick_ctr is not None else 0) \
            | (8 if zero_grad else 0)
        C().adam_step(w, g, m, v, w16, lr, beta1, beta2, eps, weight_decay, mode, bc1, bc2, grad_scale, device_step,
                      tick_ctr)
        return
    d = g * grad_scale
    if decoupled:
        w.mul_(1.0 - lr * weight_decay)
    elif weight_decay:
        d = d + weight_decay * w
    m.mul_(beta1).add_(d, alpha=1.0 - beta1)
    v.mul_(beta2).addcmul_(d, d, value=1.0 - beta2)
    if keras_eps:
        w.sub_(lr * (bc2 ** 0.5) / bc1 * m / (v.sqrt() + eps))
    else:
        w.sub_(lr * (m / bc1) / (v.sqrt() / (bc2 ** 0.5) + eps))
    if w16 is not None and w16.data_ptr() != w.data_ptr():
        w16.copy_(w)


def step_tick(device_step):
    """+1 on the device step counter (one launch per optimizer step)."""
    if use_native(device_step):
        C().step_tick(device_step)
    else:
        device_step.add_(1.0)


def adagrad_(w, g, acc, w16, *, lr, eps=1e-7, weight_decay=0.0, grad_scale=1.0):
    if use_native(w):
        C().adagrad_step(w, g, acc, w16, lr, eps, weight_decay, grad_scale)
        return
    d = g * grad_scale
    if weight_decay:
        d = d + weight_decay * w
    acc.addcmul_(d, d)
    w.sub_(lr * d / (acc.sqrt() + eps))
    if w16 is not None and w16.data_ptr() != w.data_ptr():
        w16.copy_(w)


def rmsprop_(w, g, acc, w16, *, lr, rho=0.9, eps=1e-7, weight_decay=0.0, grad_scale=1.0):
    if use_native(w):
        C().rmsprop_step(w, g, acc, w16, lr, rho, eps, weight_decay, grad_scale)
        return
    d = g * grad_scale
    if weight_decay:
        d = d + weight_decay * w
    acc.mul_(rho).addcmul_(d, d, value=1.0 - rho)
    w.sub_(lr * d / (acc.sqrt() + eps))
    if w16 is not None and w16.data_ptr() != w.data_ptr():
        w16.copy_(w)


def cast_master_to_compute(w, w16):
    if w16 is None or w16.data_ptr() == w.data_ptr():
        return
    if use_native(w) and w16.dtype == torch.bfloat16:
        C().cast_f32_bf16(w, w16)
    else:
        w16.copy_(w)
