"""Transformer ops: fused attention, LayerNorm, BERT embeddings (HIP kernels on GPU,
PyTorch reference on CPU) and the stateless dropout mask shared by both paths.

GPU kernels: ``csrc/kernels/attention.hip`` (flash-style fwd + two-kernel bwd on MFMA),
``csrc/kernels/layernorm.hip`` (LayerNorm fwd/bwd, embeddings, partial-row column sums)
and the GEMM epilogue extensions in ``csrc/include/ddl_gemm_kernel.h`` (GELU, dropout,
residual add).  The dropout mask is a hash of ``(seed, element index)``; the reference
implementation below reproduces it bit-exactly, so CPU and GPU agree even with dropout on.
"""
from __future__ import annotations

import math

import torch

from ._native import C, use_native
from ._ref import accumulate, ref_grads

def drop_hash_ref(seed: int, idx: torch.Tensor) -> torch.Tensor:
    """The dropout byte of element ``idx`` (ddl_common.h ``drop_keep``): byte ``idx % 4`` of
    ``drop_hash4(seed + idx // 4)``, on int64 tensors (values 0..255)."""
    s = seed & 0xFFFFFFFFFFFFFFFF
    if s >= 1 << 63:
        s -= 1 << 64
    idx = idx.to(torch.int64)
    q = (idx >> 2) + s  # wraps mod 2^64 like the device's uint64 add
    m = 0xFFFFFFFF
    x = (q & m) ^ ((((q >> 32) & 0xFFFFFF) * 0x9E3779) & m)
    x = (x * 0x9E3779B1) & m  # (int64 products wrap; the low 32 bits are exact)
    x = x ^ (x >> 16)
    x = ((x & 0xFFFFFF) * 0x7FEB35) & m
    x = x ^ (x >> 15)
    x = ((x & 0xFFFFFF) * 0x846CA7) & m
    x = x ^ (x >> 16)
    return (x >> (8 * (idx & 3))) & 0xFF


def drop_thresh(p: float) -> int:
    """Threshold byte of a dropout rate: the rate is quantised to 1/256 (ddl_ops.h ``drop_t8``)."""
    return min(255, max(1, math.floor(p * 256.0 + 0.5))) if p > 0 else 0


def drop_scale(p: float) -> float:
    """Scale of the kept values: the inverse of the quantised keep rate (ddl_ops.h ``drop_scale8``)."""
    t8 = drop_thresh(p)
    return 256.0 / (256.0 - t8) if t8 else 1.0


def keep_mask_ref(seed: int, idx: torch.Tensor, p: float) -> torch.Tensor:
    return drop_hash_ref(seed, idx) >= drop_thresh(p)


def dropout_ref(x: torch.Tensor, p: float, seed: int) -> torch.Tensor:
    """Dropout of a [M, N] matrix with element index m*N + n (the GEMM-epilogue convention)."""
    if p <= 0:
        return x
    idx = torch.arange(x.numel(), device=x.device).view(x.shape)
    return torch.where(keep_mask_ref(seed, idx, p), x * drop_scale(p), torch.zeros((), dtype=x.dtype, device=x.device))


# ============================================================================ attention
def mix32_ref(x: torch.Tensor) -> torch.Tensor:
    """``mix32`` of csrc/kernels/attention.hip on int64 tensors holding uint32 values."""
    m = 0xFFFFFFFF
    x = x & m
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & m
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & m
    return x ^ (x >> 16)


def hash24_ref(x: torch.Tensor) -> torch.Tensor:
    """``hash24`` of csrc/kernels/attention.hip: the 32-bit mix with 24-bit multiplies (v_mul_u32_u24)."""
    m = 0xFFFFFFFF
    x = x & m
    x = x ^ (x >> 16)
    x = ((x & 0xFFFFFF) * 0x7FEB35) & m
    x = x ^ (x >> 15)
    x = ((x & 0xFFFFFF) * 0x846CA7) & m
    return x ^ (x >> 16)


def attn_drop_t8(p: float) -> int:
    """Attention dropout threshold byte (the same quantisation as every dropout here: drop_thresh)."""
    return drop_thresh(p)


def attn_drop_scale(p: float) -> float:
    """Scale of the kept attention probabilities: the inverse of the quantised keep rate."""
    return drop_scale(p)


def attn_keep_ref(seed: int, row: torch.Tensor, j: torch.Tensor, p: float) -> torch.Tensor:
    """Attention-probability dropout mask.  One 32-bit hash h = hash24(row_key(row) + j // 4)
    serves four consecutive keys: key j keeps iff byte j % 4 of h is >= attn_drop_t8(p), with
    row_key = mix32(seed_lo ^ mix32(row + seed_hi)) and row = (b*H + h)*S + i."""
    s = seed & 0xFFFFFFFFFFFFFFFF
    lo, hi = s & 0xFFFFFFFF, s >> 32
    rk = mix32_ref(lo ^ mix32_ref(row.to(torch.int64) + hi))
    j = j.to(torch.int64)
    h = hash24_ref(rk + (j >> 2))
    return ((h >> (8 * (j & 3))) & 0xFF) >= attn_drop_t8(p)


def attention_ref(qkv, B, S, H, q_off, k_off, v_off, lens=None, scale=0.125, drop_p=0.0, seed=0):
    """fp32 reference: qkv [B*S, W] -> context [B*S, H*64]."""
    x = qkv.float().view(B, S, -1)

    def heads(off):
        return x[..., off : off + H * 64].view(B, S, H, 64).permute(0, 2, 1, 3)

    q, k, v = heads(q_off), heads(k_off), heads(v_off)
    s = torch.einsum("bhid,bhjd->bhij", q, k) * scale
    if lens is not None:
        key_ok = torch.arange(S, device=qkv.device)[None, :] < lens.to(qkv.device).long()[:, None]
        s = s.masked_fill(~key_ok[:, None, None, :], float("-inf"))
    p = torch.softmax(s, dim=-1)
    if lens is not None:
        p = torch.nan_to_num(p, nan=0.0)
    if drop_p > 0:
        bh = torch.arange(B * H, device=qkv.device).view(B, H, 1, 1)
        i = torch.arange(S, device=qkv.device).view(1, 1, S, 1)
        j = torch.arange(S, device=qkv.device).view(1, 1, 1, S)
        keep = attn_keep_ref(seed, bh * S + i, j, drop_p)
        p = torch.where(keep, p * attn_drop_scale(drop_p), torch.zeros((), device=p.device))
    o = torch.einsum("bhij,bhjd->bhid", p, v)
    return o.permute(0, 2, 1, 3).reshape(B * S, H * 64)


class _AttentionFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cfg):
        B, S, H, offs, lens, scale, drop_p, seed = cfg
        ctx.cfg = cfg
        if use_native(qkv):
            o = torch.empty((B * S, H * 64), dtype=torch.bfloat16, device=qkv.device)
            lse = torch.empty((B, H, S), dtype=torch.float32, device=qkv.device)
            C().attn_fwd(qkv, B, S, H, *offs, o, lse, lens, scale, drop_p, seed)
            ctx.save_for_backward(qkv, o, lse)
            ctx.native = True
            return o
        ctx.native = False
        ctx.save_for_backward(qkv)
        return attention_ref(qkv, B, S, H, *offs, lens, scale, drop_p, seed).to(qkv.dtype)

    @staticmethod
    def backward(ctx, do):
        B, S, H, offs, lens, scale, drop_p, seed = ctx.cfg
        if ctx.native:
            qkv, o, lse = ctx.saved_tensors
            # the dQ / dK / dV kernels store every row of their head columns (S % 128 == 0, unmasked
            # stores), so a packed [tokens, 3*H*64] QKV needs no zero fill (a 75 MB fill per BERT-base
            # layer); other layouts keep zeros in the columns no head owns
            HD = H * 64
            packed = tuple(offs) == (0, HD, 2 * HD) and qkv.shape[1] == 3 * HD and qkv.is_contiguous()
            dqkv = torch.empty_like(qkv) if packed else torch.zeros_like(qkv)
            dvec = torch.empty((B, H, S), dtype=torch.float32, device=qkv.device)
            C().attn_bwd(qkv, B, S, H, *offs, o, lse, lens, scale, drop_p, seed, do.contiguous(), dvec, dqkv)
            return dqkv, None
        (qkv,) = ctx.saved_tensors
        (g,) = ref_grads(lambda t: attention_ref(t, B, S, H, *offs, lens, scale, drop_p, seed), [qkv], do.float())
        return g.to(qkv.dtype), None


def attention(qkv, B, S, H, *, q_off=None, k_off=None, v_off=None, lens=None, scale=None, drop_p=0.0, seed=0):
    """Multi-head attention over a packed ``[B*S, 3*H*64]`` QKV projection (head dim 64)."""
    HD = H * 64
    offs = (0 if q_off is None else q_off, HD if k_off is None else k_off, 2 * HD if v_off is None else v_off)
    scale = 1.0 / math.sqrt(64) if scale is None else scale
    if lens is not None:
        lens = lens.to(torch.int32).contiguous()
    return _AttentionFn.apply(qkv, (B, S, H, offs, lens, float(scale), float(drop_p), int(seed)))


# ============================================================================ LayerNorm
def layer_norm_ref(x, gamma, beta, eps):
    return torch.nn.functional.layer_norm(x.float(), (x.shape[-1],), None if gamma is None else gamma.float(),
                                          None if beta is None else beta.float(), eps)


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, gamma, beta, gg, gb, eps, hook):
        ctx.eps, ctx.hook, ctx.gg, ctx.gb = eps, hook, gg, gb
        ctx.native = use_native(x)
        H = x.shape[-1]
        if ctx.native:
            x2 = x.reshape(-1, H).contiguous()
            M = x2.shape[0]
            y = torch.empty_like(x2)
            mean = torch.empty(M, dtype=torch.float32, device=x.device)
            rstd = torch.empty_like(mean)
            C().layernorm_fwd(x2, gamma, beta, y, mean, rstd, eps)
            ctx.save_for_backward(x2, mean, rstd)
            ctx.gamma = gamma
            ctx.shape = x.shape
            return y.view(x.shape)
        ctx.save_for_backward(x, gamma, beta)
        return layer_norm_ref(x, gamma, beta, eps).to(x.dtype)

    @staticmethod
    def backward(ctx, dy):
        if ctx.native:
            x2, mean, rstd = ctx.saved_tensors
            H = x2.shape[-1]
            M = x2.shape[0]
            dx = torch.empty_like(x2)
            ws = None
            if ctx.gg is not None or ctx.gb is not None:
                P = C().ln_bwd_rows(M, H)
                ws = torch.empty((P, 2, H), dtype=torch.float32, device=x2.device)
            C().layernorm_bwd(dy.reshape(-1, H).contiguous(), x2, mean, rstd, ctx.gamma, dx, None, 0.0, 0, ws)
            if ws is not None:
                wsv = ws.view(-1, 2 * H)
                red = torch.empty(2 * H, dtype=torch.float32, device=x2.device)
                C().colsum_partials(wsv, wsv.shape[0], 2 * H, red, False)
                if ctx.gg is not None:
                    ctx.gg.add_(red[:H])
                if ctx.gb is not None:
                    ctx.gb.add_(red[H:])
            out = dx.view(ctx.shape)
        else:
            x, gamma, beta = ctx.saved_tensors
            gx, gg, gbb = ref_grads(lambda a, g, b: layer_norm_ref(a, g, b, ctx.eps), [x, gamma, beta], dy.float())
            accumulate(ctx.gg, gg)
            accumulate(ctx.gb, gbb)
            out = gx.to(x.dtype)
        if ctx.hook is not None:
            ctx.hook()
        return out, None, None, None, None, None, None, None


def layer_norm(x, gamma=None, beta=None, eps=1e-12, *, grad_gamma=None, grad_beta=None, anchor=None, on_grad=None):
    """LayerNorm over the last dim; fp32 gamma/beta (the arena masters), out-of-band grads."""
    if anchor is None:
        anchor = gamma if gamma is not None else x
    return _LayerNormFn.apply(x, anchor, gamma, beta, grad_gamma, grad_beta, float(eps), on_grad)
