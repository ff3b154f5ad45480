"""Batch normalisation (NHWC, training statistics) with fused residual-add + ReLU.

GPU path (csrc/kernels/bn.hip): statistics either come fused from the producing
convolution's epilogue (``stats`` workspace filled by the GEMM) or from one
``bn_stats`` sweep; a per-channel finalize yields scale/shift and updates running
statistics; one apply sweep writes ``relu(x*scale + shift + residual)``.  Backward is
reduce (masked dy, dy*xhat) -> finalize (dgamma/dbeta, coefficients) -> one dx sweep that
also emits the masked gradient of the residual branch.
"""
from __future__ import annotations

import torch

from . import determinism as _det
from . import scope as _scope
from ._native import C, use_native
from ._ref import accumulate, ref_grads

SHARDS = 32


class _StatsPool:
    """Bump allocator for the per-layer [SHARDS, 2, C] statistics workspaces.

    One zeroing memset per training step (``reset``) replaces ~2 small memset
    launches per BN layer; the buffer grows to the largest per-step demand seen."""

    def __init__(self):
        self.buf, self.used, self.demand = {}, {}, {}

    @staticmethod
    def _key(device):
        d = torch.device(device)
        if d.type == "cuda" and d.index is None:  # "cuda" and "cuda:0" must share one pool entry
            d = torch.device("cuda", torch.cuda.current_device())
        return str(d) + _scope.tag()

    def get(self, C_, device):
        key = self._key(device)
        n = -(-SHARDS * 2 * C_ // 64) * 64
        self.demand[key] = self.demand.get(key, 0) + n
        buf, used = self.buf.get(key), self.used.get(key, 0)
        if buf is None or used + n > buf.numel():
            return torch.zeros((SHARDS, 2, C_), dtype=torch.float32, device=device)
        self.used[key] = used + n
        return buf[used : used + SHARDS * 2 * C_].view(SHARDS, 2, C_)

    def reset(self, device):
        """Start a new step: returns the part of the pool the last step used (to be zeroed by the caller),
        or None (nothing used, or a freshly zero-allocated pool sized to the last step's demand)."""
        key = self._key(device)
        want = self.demand.get(key, 0)
        buf = self.buf.get(key)
        dirty = None
        if want and (buf is None or buf.numel() < want):
            self.buf[key] = torch.zeros(want, dtype=torch.float32, device=device)
        elif buf is not None and self.used.get(key, 0):
            dirty = buf[: self.used[key]]
        self.used[key] = 0
        self.demand[key] = 0
        return dirty


_POOL = _StatsPool()


def new_stats_workspace(C_, device):
    """[32, 2, C] zeroed workspace for statistics fused into a GEMM epilogue (atomic shards), or None in
    the deterministic mode: the consumer then runs the fixed-order ``bn_stats`` sweep instead."""
    if _det.enabled():
        return None
    if torch.device(device).type == "cuda":
        return _POOL.get(C_, device)
    return torch.zeros((SHARDS, 2, C_), dtype=torch.float32, device=device)


def partials_workspace(M, C_, device):
    """[S, 2, C] partial-sum rows written (not accumulated) by a bn_stats / bn_bwd_reduce sweep."""
    return torch.empty((C().bn_partial_rows(M, C_), 2, C_), dtype=torch.float32, device=device)


def reset_workspaces(device, extra=None):
    """Call once per training step before the forward: zeroes the statistics workspaces and ``extra``
    (the gradient arena, when the step needs it zeroed) in ONE launch (``zero_ranges``)."""
    dirty = _POOL.reset(device) if torch.device(device).type == "cuda" else None
    bufs = [t for t in (dirty, extra) if t is not None and t.numel()]
    if not bufs:
        return
    if bufs[0].is_cuda:
        C().zero_ranges(bufs)
    else:
        for t in bufs:
            t.zero_()


def bn_ref(x, gamma, beta, mean, var, eps, resid=None, relu=False):
    y = (x - mean) / torch.sqrt(var + eps)
    if gamma is not None:
        y = y * gamma
    if beta is not None:
        y = y + beta
    if resid is not None:
        y = y + resid
    if relu:
        y = torch.relu(y)
    return y


def _bn_train_ref(x, gamma, beta, eps, resid, relu):
    dims = tuple(range(x.dim() - 1))
    mean = x.mean(dims)
    var = x.var(dims, unbiased=False)
    return bn_ref(x, gamma, beta, mean, var, eps, resid, relu)


class _BatchNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, resid, ggamma, gbeta, state):
        rmean, rvar, momentum, eps, relu, training, stats, hook = state
        Cc = x.shape[-1]
        M = x.numel() // Cc
        ctx.native = use_native(x)
        ctx.relu, ctx.eps, ctx.hook, ctx.training = relu, eps, hook, training
        ctx.has_resid = resid is not None
        if ctx.native:
            x = x.contiguous()
            dev = x.device
            scale = torch.empty(Cc, dtype=torch.float32, device=dev)
            shift = torch.empty(Cc, dtype=torch.float32, device=dev)
            mean = torch.empty(Cc, dtype=torch.float32, device=dev)
            invstd = torch.empty(Cc, dtype=torch.float32, device=dev)
            if training:
                if stats is None:
                    stats = partials_workspace(M, Cc, dev)
                    C().bn_stats(x, stats, Cc)
                C().bn_finalize(stats, M, Cc, gamma, beta, eps, momentum, rmean, rvar, mean, invstd, scale, shift)
            else:
                invstd = torch.rsqrt(rvar + eps)
                mean = rmean.clone()
                g = gamma if gamma is not None else torch.ones_like(rmean)
                b = beta if beta is not None else torch.zeros_like(rmean)
                scale = (g * invstd).contiguous()
                shift = (b - rmean * scale).contiguous()
            y = torch.empty_like(x)
            C().bn_apply(x, scale, shift, None if resid is None else resid.contiguous(), y, Cc, relu, None)
            ctx.gg, ctx.gbt = ggamma, gbeta
            # relu mask for backward: recompute from x*scale+shift (no resid) or read y (resid)
            ctx.mode = 0 if not relu else (1 if resid is not None else 2)
            ctx.save_for_backward(x, y if ctx.mode == 1 else None, mean, invstd, gamma, scale, shift)
            return y
        # reference path
        if training:
            dims = tuple(range(x.dim() - 1))
            with torch.no_grad():
                bm = x.mean(dims)
                bv = x.var(dims, unbiased=False)
                if rmean is not None:
                    n = x.numel() // Cc
                    rmean.mul_(1 - momentum).add_(momentum * bm.to(rmean.dtype))
                    rvar.mul_(1 - momentum).add_(momentum * (bv * n / max(n - 1, 1)).to(rvar.dtype))
            y = _bn_train_ref(x, gamma, beta, eps, resid, relu)
        else:
            y = bn_ref(x, gamma, beta, rmean, rvar, eps, resid, relu)
        ctx.gg, ctx.gbt, ctx.rstats = ggamma, gbeta, (rmean, rvar)
        ctx.save_for_backward(x, resid, gamma, beta)
        return y

    @staticmethod
    def backward(ctx, dy):
        dres = None
        if ctx.native:
            x, y, mean, invstd, gamma, scale, shift = ctx.saved_tensors
            ggamma, gbeta = ctx.gg, ctx.gbt
            dy = dy.contiguous()
            Cc = x.shape[-1]
            M = x.numel() // Cc
            if not ctx.training:  # eval-mode statistics are constants: dx = dy' * gamma * invstd
                d = dy.float()
                if ctx.mode:
                    d = d * ((x.float() * scale + shift) > 0) if y is None else d * (y.float() > 0)
                xh = (x.float() - mean) * invstd
                dims = tuple(range(x.dim() - 1))
                if ggamma is not None:
                    ggamma.add_((d * xh).sum(dims))
                if gbeta is not None:
                    gbeta.add_(d.sum(dims))
                dx = (d * scale).to(x.dtype)
                dres = d.to(x.dtype) if ctx.has_resid else None
            else:
                ws = partials_workspace(M, Cc, x.device)
                C().bn_bwd_reduce(dy, x, y, scale, shift, mean, ws, Cc, ctx.mode)
                coef = torch.empty(3 * Cc, dtype=torch.float32, device=x.device)
                C().bn_bwd_finalize(ws, M, Cc, gamma, mean, invstd, ggamma, gbeta, coef)
                dx = torch.empty_like(x)
                if ctx.has_resid:
                    dres = torch.empty_like(x)
                C().bn_bwd_dx(dy, x, y, scale, shift, coef, dx, dres, Cc, ctx.mode)
        else:
            x, resid, gamma, beta = ctx.saved_tensors
            ggamma, gbeta = ctx.gg, ctx.gbt
            rmean, rvar = ctx.rstats
            eps, relu = ctx.eps, ctx.relu
            if ctx.training:
                fn = lambda xx, gg, bb, rr: _bn_train_ref(xx, gg, bb, eps, rr, relu)
            else:
                fn = lambda xx, gg, bb, rr: bn_ref(xx, gg, bb, rmean, rvar, eps, rr, relu)
            dx, dg, db, dres = ref_grads(fn, [x, gamma, beta, resid], dy)
            accumulate(ggamma, dg)
            accumulate(gbeta, db)
        if ctx.hook is not None:
            ctx.hook()
        return dx, None, None, dres, None, None, None


def batch_norm(x, gamma, beta, running_mean, running_var, *, training=True, momentum=0.1, eps=1e-5, resid=None,
               relu=False, grad_gamma=None, grad_beta=None, stats=None, on_grad=None):
    """NHWC batch norm over all but the last dim.  ``stats``: fused statistics workspace
    already accumulated by the producer (GPU); ``resid``/``relu``: fused epilogue."""
    state = (running_mean, running_var, momentum, eps, bool(relu), bool(training), stats, on_grad)
    return _BatchNormFn.apply(x, gamma, beta, resid, grad_gamma, grad_beta, state)
