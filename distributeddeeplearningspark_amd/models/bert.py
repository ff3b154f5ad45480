"""BERT (post-LayerNorm encoder) with the masked-LM head — the BASELINE.json
"BERT-base MLM seq-len 512" configuration.

GPU execution (one autograd node per encoder layer, backward scheduled by hand):

  qkv  = h Wqkv^T + b                       GEMM, bias epilogue            [T, 3H]
  ctx  = attention(qkv)                     fused MFMA attention (prob. dropout in-kernel)
  s1   = h + dropout(ctx Wo^T + bo)         GEMM epilogue: bias, dropout, residual add
  a    = LN1(s1)
  f    = gelu(a W1^T + b1)                  GEMM epilogue: bias, GELU (pre-activation kept)
  s2   = a + dropout(f W2^T + b2)           GEMM epilogue
  h'   = LN2(s2)

Backward: LN2' emits both d(s2) and the dropout-masked gradient of the FFN output in one
pass; the W2 data-gradient GEMM multiplies by gelu'(pre) in its epilogue; the W1 data
gradient adds the residual gradient in its epilogue; the same for the attention block.
No elementwise kernels remain between GEMMs.  Parameter gradients go straight into the
flat fp32 gradient arena (wgrad GEMMs accumulate with beta = 1), and each layer fires its
data-parallel grad hook when its gradients are final.

Masked-LM loss: only the masked positions (``masked_lm_positions``, padded to
``max_predictions_per_seq`` with label -100) go through the transform + decoder
(decoder weight tied to the word embeddings; the vocabulary is stored padded to a
multiple of 8 rows so every GEMM operand row is 16-B aligned).  The loss equals the
full-sequence masked CE (non-masked positions contribute nothing to it).

CPU: the same math from stock PyTorch ops (fp32) with the SAME hash dropout masks,
used by the tests as the numerics reference of the GPU path.
"""
from __future__ import annotations

import math
from dataclasses import asdict, dataclass

import numpy as np
import torch
import torch.nn.functional as F

from ..ops import determinism as _det
from ..ops import gemm as G
from ..ops import transformer as T
from ..ops._native import C, use_native
from ..ops.norm import new_stats_workspace
from ..ops._ref import ref_grads
from ..ops.streams import on_grad_stream
from . import params as P
from .core import Layer, Model


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.1
    layer_norm_eps: float = 1e-12
    initializer_range: float = 0.02

    @property
    def vocab_padded(self) -> int:
        return -(-self.vocab_size // 8) * 8

    @staticmethod
    def base(**kw):
        return BertConfig(**kw)

    @staticmethod
    def tiny(**kw):
        d = dict(vocab_size=1000, hidden_size=128, num_hidden_layers=2, num_attention_heads=2, intermediate_size=512,
                 max_position_embeddings=256)
        d.update(kw)
        return BertConfig(**d)


_MASK64 = (1 << 64) - 1


def _seed(*parts) -> int:
    h = 0x9E3779B97F4A7C15
    for p in parts:
        h = ((h ^ (int(p) & _MASK64)) * 0xBF58476D1CE4E5B9) & _MASK64
        h ^= h >> 31
    return h & 0x7FFFFFFFFFFFFFFF


def _contiguous(*ts) -> bool:
    """True when the 1-D tensors are back-to-back in memory (consecutive arena parameters)."""
    for a, b in zip(ts, ts[1:]):
        if a.data_ptr() + a.numel() * a.element_size() != b.data_ptr():
            return False
    return True


def _ln_param_grads(ws, H, g_param, b_param):
    """Column sums of LayerNorm partial rows [P][2][H] into (gamma, beta) gradients."""
    P_ = ws.shape[0]
    if _contiguous(g_param.grad, b_param.grad):
        C().colsum_partials(ws.view(P_, 2 * H), P_, 2 * H, g_param.grad.as_strided((2 * H,), (1,)), True)
    else:
        red = torch.empty(2 * H, dtype=torch.float32, device=ws.device)
        C().colsum_partials(ws.view(P_, 2 * H), P_, 2 * H, red, False)
        g_param.grad.add_(red[:H])
        b_param.grad.add_(red[H:])


def _bias_grad(d2, gb):
    if gb is not None:
        C().bias_grad(d2, gb, d2.shape[1], True)


# Every BERT GEMM (fused-epilogue or plain) runs on the hand-written MFMA kernels; the
# hipBLASLt route tried in round 1 measured slower end-to-end and was removed (PERFORMANCE.md).
def _wgrad(d2, x2, gw):
    # weight gradients run on the side stream beside the data-gradient chain (ops/streams.py)
    with on_grad_stream(d2.device, d2, x2):
        G.linear_wgrad(d2, x2, gw)


def _dgrad(dy, w):
    return G.linear_dgrad(dy, w)


# ====================================================================================== layers
class BertEmbeddings(Layer):
    def __init__(self, cfg: BertConfig, **kw):
        super().__init__(**kw)
        self.cfg = cfg

    def build(self, s):
        c = self.cfg
        init = P.truncated_normal(c.initializer_range)

        def word_init(shape, gen):
            w = init(shape, gen)
            w[c.vocab_size:] = 0.0  # padding rows (never looked up, zero logits weight)
            return w

        self.word = self.add_weight("word_embeddings", (c.vocab_padded, c.hidden_size), word_init)
        self.pos = self.add_weight("position_embeddings", (c.max_position_embeddings, c.hidden_size), init)
        self.type = self.add_weight("token_type_embeddings", (c.type_vocab_size, c.hidden_size), init)
        self.ln_g = self.add_weight("LayerNorm/gamma", (c.hidden_size,), P.ones)
        self.ln_b = self.add_weight("LayerNorm/beta", (c.hidden_size,), P.zeros)
        return s


class BertLayer(Layer):
    def __init__(self, cfg: BertConfig, index: int, **kw):
        super().__init__(**kw)
        self.cfg, self.index = cfg, index

    def build(self, s):
        c = self.cfg
        H, I = c.hidden_size, c.intermediate_size
        init = P.truncated_normal(c.initializer_range)
        self.qkv_w = self.add_weight("attention/qkv/kernel", (3 * H, H), init)
        self.qkv_b = self.add_weight("attention/qkv/bias", (3 * H,), P.zeros)
        self.o_w = self.add_weight("attention/output/kernel", (H, H), init)
        self.o_b = self.add_weight("attention/output/bias", (H,), P.zeros)
        self.ln1_g = self.add_weight("attention/LayerNorm/gamma", (H,), P.ones)
        self.ln1_b = self.add_weight("attention/LayerNorm/beta", (H,), P.zeros)
        self.i_w = self.add_weight("intermediate/kernel", (I, H), init)
        self.i_b = self.add_weight("intermediate/bias", (I,), P.zeros)
        self.out_w = self.add_weight("output/kernel", (H, I), init)
        self.out_b = self.add_weight("output/bias", (H,), P.zeros)
        self.ln2_g = self.add_weight("output/LayerNorm/gamma", (H,), P.ones)
        self.ln2_b = self.add_weight("output/LayerNorm/beta", (H,), P.zeros)
        return s


class BertMLMHead(Layer):
    def __init__(self, cfg: BertConfig, **kw):
        super().__init__(**kw)
        self.cfg = cfg

    def build(self, s):
        c = self.cfg
        H = c.hidden_size
        self.t_w = self.add_weight("transform/dense/kernel", (H, H), P.truncated_normal(c.initializer_range))
        self.t_b = self.add_weight("transform/dense/bias", (H,), P.zeros)
        self.ln_g = self.add_weight("transform/LayerNorm/gamma", (H,), P.ones)
        self.ln_b = self.add_weight("transform/LayerNorm/beta", (H,), P.zeros)
        self.dec_b = self.add_weight("decoder/bias", (c.vocab_padded,), P.zeros)
        return s


# ====================================================================================== reference math
def _ln(x, g, b, eps):
    return F.layer_norm(x, (x.shape[-1],), g, b, eps)


def _drop2d(x, p, seed):
    return T.dropout_ref(x, p, seed) if p > 0 else x


def embeddings_ref(ids, types, word, pos, typ, g, b, eps, p, seed, S):
    T_ = ids.numel()
    pos_idx = torch.arange(T_, device=ids.device) % S
    e = word[ids.reshape(-1)] + pos[pos_idx] + typ[(types.reshape(-1) if types is not None else torch.zeros_like(
        ids.reshape(-1)))]
    return _drop2d(_ln(e, g, b, eps), p, seed)


def layer_ref(h, w, cfg: BertConfig, B, S, lens, p_h, p_a, seeds):
    """One post-LN encoder layer in fp32 (w: dict of fp32 weights)."""
    H, NH, eps = cfg.hidden_size, cfg.num_attention_heads, cfg.layer_norm_eps
    qkv = h @ w["qkv_w"].t() + w["qkv_b"]
    ctx = T.attention_ref(qkv, B, S, NH, 0, H, 2 * H, lens, 1.0 / math.sqrt(64), p_a, seeds[0])
    s1 = h + _drop2d(ctx @ w["o_w"].t() + w["o_b"], p_h, seeds[1])
    a = _ln(s1, w["ln1_g"], w["ln1_b"], eps)
    f = F.gelu(a @ w["i_w"].t() + w["i_b"])
    s2 = a + _drop2d(f @ w["out_w"].t() + w["out_b"], p_h, seeds[2])
    return _ln(s2, w["ln2_g"], w["ln2_b"], eps)


def mlm_head_ref(hm, t_w, t_b, g, b, word, dec_b, eps, V):
    t = _ln(F.gelu(hm @ t_w.t() + t_b), g, b, eps)
    return t @ word[:V].t() + dec_b[:V]


_LAYER_KEYS = ("qkv_w", "qkv_b", "o_w", "o_b", "ln1_g", "ln1_b", "i_w", "i_b", "out_w", "out_b", "ln2_g", "ln2_b")


# ====================================================================================== autograd nodes
class _EmbeddingsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, layer, ids, types, S, p, seed):
        c = layer.cfg
        ctx.layer, ctx.S, ctx.p, ctx.seed = layer, S, p, seed
        ctx.native = use_native(anchor)
        if ctx.native:
            T_ = ids.numel()
            H = c.hidden_size
            e = torch.empty((T_, H), dtype=torch.bfloat16, device=anchor.device)
            C().embed_fwd(ids.reshape(-1), None if types is None else types.reshape(-1), layer.word.data,
                          layer.pos.data, layer.type.data, e, S)
            y = torch.empty_like(e)
            mean = torch.empty(T_, dtype=torch.float32, device=e.device)
            rstd = torch.empty_like(mean)
            C().layernorm_fwd(e, layer.ln_g.master, layer.ln_b.master, y, mean, rstd, c.layer_norm_eps, p, seed)
            ctx.save_for_backward(ids, types, e, mean, rstd)
            return y
        ctx.save_for_backward(ids, types)
        with torch.no_grad():
            return embeddings_ref(ids, types, layer.word.master, layer.pos.master, layer.type.master,
                                  layer.ln_g.master, layer.ln_b.master, c.layer_norm_eps, p, seed, S)

    @staticmethod
    def backward(ctx, dy):
        layer, S = ctx.layer, ctx.S
        c = layer.cfg
        H = c.hidden_size
        if ctx.native:
            ids, types, e, mean, rstd = ctx.saved_tensors
            T_ = e.shape[0]
            de = torch.empty_like(e)
            ws = torch.empty((C().ln_bwd_rows(T_, H), 2, H), dtype=torch.float32, device=e.device)
            C().layernorm_bwd(dy.contiguous(), e, mean, rstd, layer.ln_g.master, de, None, 0.0, 0, ws, ctx.p, ctx.seed)
            _ln_param_grads(ws, H, layer.ln_g, layer.ln_b)
            # word rows: no-return fp32 atomics straight into the arena (no id sort); positions: sum over batch
            # (side stream: ordered after the tied decoder's wgrad into the same rows)
            with on_grad_stream(de.device, de, ids):
                if _det.enabled():  # stable id sort + one writer per run of equal ids (fixed order)
                    sids, perm = torch.sort(ids.reshape(-1), stable=True)
                    C().embed_word_grad_det(sids, perm, de, layer.word.grad)
                else:
                    C().embed_word_grad_atomic(ids.reshape(-1).contiguous(), de, layer.word.grad)
            C().embed_pos_grad(de, layer.pos.grad, T_ // S, S)
            nt = c.type_vocab_size
            if nt <= 2:
                P_ = C().embed_partial_rows(T_)
                wsT = torch.empty((P_, nt, H), dtype=torch.float32, device=e.device)
                C().embed_bwd(ids.reshape(-1), None if types is None else types.reshape(-1), de, None, None, wsT, nt,
                              S)
                C().colsum_partials(wsT.view(P_, nt * H), P_, nt * H, layer.type.grad.view(-1), True)
            else:
                tt = types.reshape(-1) if types is not None else torch.zeros(T_, dtype=torch.long, device=e.device)
                layer.type.grad.index_add_(0, tt, de.float())
        else:
            ids, types = ctx.saved_tensors
            ws = [layer.word.master, layer.pos.master, layer.type.master, layer.ln_g.master, layer.ln_b.master]
            grads = ref_grads(lambda w_, p_, t_, g_, b_: embeddings_ref(ids, types, w_, p_, t_, g_, b_,
                                                                        c.layer_norm_eps, ctx.p, ctx.seed, S),
                              ws, dy.float())
            for prm, g in zip((layer.word, layer.pos, layer.type, layer.ln_g, layer.ln_b), grads):
                prm.grad.add_(g)
        if layer.grad_hook is not None:
            layer.grad_hook()
        return None, None, None, None, None, None, None


class _BertLayerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, anchor, layer, B, S, lens, p_h, p_a, seeds):
        c = layer.cfg
        ctx.layer, ctx.B, ctx.S, ctx.lens, ctx.p_h, ctx.p_a, ctx.seeds = layer, B, S, lens, p_h, p_a, seeds
        ctx.native = use_native(h)
        H, NH, eps = c.hidden_size, c.num_attention_heads, c.layer_norm_eps
        if not ctx.native:
            ctx.save_for_backward(h)
            w = {k: getattr(layer, k).master for k in _LAYER_KEYS}
            with torch.no_grad():
                return layer_ref(h.float(), w, c, B, S, lens, p_h, p_a, seeds).to(h.dtype)
        L = layer
        T_ = h.shape[0]
        dev = h.device
        qkv = G.linear_fwd(h, L.qkv_w.data, bias=L.qkv_b.master)
        ctxo = torch.empty((T_, H), dtype=torch.bfloat16, device=dev)
        lse = torch.empty((B, NH, S), dtype=torch.float32, device=dev)
        C().attn_fwd(qkv, B, S, NH, 0, H, 2 * H, ctxo, lse, lens, 1.0 / math.sqrt(64), p_a, seeds[0])
        s1 = G.linear_fwd(ctxo, L.o_w.data, bias=L.o_b.master, resid=h, drop_p=p_h, drop_seed=seeds[1])
        a = torch.empty_like(s1)
        m1 = torch.empty(T_, dtype=torch.float32, device=dev)
        r1 = torch.empty_like(m1)
        C().layernorm_fwd(s1, L.ln1_g.master, L.ln1_b.master, a, m1, r1, eps)
        pre = torch.empty((T_, c.intermediate_size), dtype=torch.bfloat16, device=dev)
        f = G.linear_fwd(a, L.i_w.data, bias=L.i_b.master, act=G.ACT_GELU, aux=pre)
        s2 = G.linear_fwd(f, L.out_w.data, bias=L.out_b.master, resid=a, drop_p=p_h, drop_seed=seeds[2])
        out = torch.empty_like(s2)
        m2 = torch.empty_like(m1)
        r2 = torch.empty_like(m1)
        C().layernorm_fwd(s2, L.ln2_g.master, L.ln2_b.master, out, m2, r2, eps)
        ctx.save_for_backward(h, qkv, ctxo, lse, s1, a, m1, r1, pre, f, s2, m2, r2)
        return out

    @staticmethod
    def backward(ctx, dout):
        L = ctx.layer
        c = L.cfg
        B, S, lens, p_h, p_a, seeds = ctx.B, ctx.S, ctx.lens, ctx.p_h, ctx.p_a, ctx.seeds
        H, NH = c.hidden_size, c.num_attention_heads
        if not ctx.native:
            (h,) = ctx.saved_tensors
            names = list(_LAYER_KEYS)
            ws = [getattr(L, k).master for k in names]
            grads = ref_grads(lambda hh, *w: layer_ref(hh, dict(zip(names, w)), c, B, S, lens, p_h, p_a, seeds),
                              [h.float()] + ws, dout.float())
            for k, g in zip(names, grads[1:]):
                getattr(L, k).grad.add_(g)
            if L.grad_hook is not None:
                L.grad_hook()
            return grads[0].to(h.dtype), None, None, None, None, None, None, None, None
        h, qkv, ctxo, lse, s1, a, m1, r1, pre, f, s2, m2, r2 = ctx.saved_tensors
        T_ = h.shape[0]
        dev = h.device
        dout = dout.contiguous()
        P_ = C().ln_bwd_rows(T_, H)
        ws = torch.empty((P_, 3, H), dtype=torch.float32, device=dev)
        red = torch.empty(3 * H, dtype=torch.float32, device=dev)

        def ln_back(dy, x, m, r, g_param, b_param, dseed, bias_param):
            """LN backward; the same sweep emits the dropout-masked gradient of the residual
            branch and its column sums (= the branch GEMM's bias gradient).  Partial rows are
            [dbias | dgamma | dbeta], the arena order of (bias, gamma, beta), so one column-sum
            launch accumulates straight into the gradient arena."""
            dx = torch.empty_like(x)
            dxd = torch.empty_like(x) if p_h > 0 else None
            C().layernorm_bwd(dy, x, m, r, g_param.master, dx, dxd, p_h, dseed, ws, 0.0, 0, 3)
            if _contiguous(bias_param.grad, g_param.grad, b_param.grad):
                span = bias_param.grad.as_strided((3 * H,), (1,))  # [bias | gamma | beta] of the arena
                C().colsum_partials(ws.view(-1, 3 * H), P_, 3 * H, span, True)
            else:
                C().colsum_partials(ws.view(-1, 3 * H), P_, 3 * H, red, False)
                bias_param.grad.add_(red[:H])
                g_param.grad.add_(red[H : 2 * H])
                b_param.grad.add_(red[2 * H :])
            return dx, (dxd if dxd is not None else dx)

        # ---- FFN block
        ds2, ds2d = ln_back(dout, s2, m2, r2, L.ln2_g, L.ln2_b, seeds[2], L.out_b)
        _wgrad(ds2d, f, L.out_w.grad)
        if _det.enabled():  # deterministic mode: no atomic epilogue statistics; one-writer column sums
            dpre = G.linear_dgrad(ds2d, L.out_w.data, gelu_pre=pre)
            _wgrad(dpre, a, L.i_w.grad)
            _bias_grad(dpre, L.i_b.grad)
        else:
            st = new_stats_workspace(c.intermediate_size, dev)  # pooled, zeroed with the step's other workspaces
            # d(pre) = (ds2d W2) * gelu'(pre); its column sums (bias grad of W1) come from the epilogue statistics
            dpre = G.linear_dgrad(ds2d, L.out_w.data, gelu_pre=pre, stats=st)
            _wgrad(dpre, a, L.i_w.grad)
            C().colsum_partials(st.view(32, -1), 32, c.intermediate_size, L.i_b.grad, True, 2 * c.intermediate_size)
        da = G.linear_dgrad(dpre, L.i_w.data, resid=ds2)  # + residual gradient
        # ---- attention block
        ds1, ds1d = ln_back(da, s1, m1, r1, L.ln1_g, L.ln1_b, seeds[1], L.o_b)
        _wgrad(ds1d, ctxo, L.o_w.grad)
        dctx = _dgrad(ds1d, L.o_w.data)
        dqkv = torch.empty_like(qkv)
        dvec = torch.empty((B, NH, S), dtype=torch.float32, device=dev)
        C().attn_bwd(qkv, B, S, NH, 0, H, 2 * H, ctxo, lse, lens, 1.0 / math.sqrt(64), p_a, seeds[0], dctx, dvec,
                     dqkv)
        _wgrad(dqkv, h, L.qkv_w.grad)
        _bias_grad(dqkv, L.qkv_b.grad)
        dh = G.linear_dgrad(dqkv, L.qkv_w.data, resid=ds1)
        if L.grad_hook is not None:
            L.grad_hook()
        return dh, None, None, None, None, None, None, None, None


class _MLMHeadFn(torch.autograd.Function):
    """Transform + tied decoder + masked softmax-CE; the loss gradient is produced in the
    forward sweep of the fused xent kernel (1/n_valid folded in)."""

    @staticmethod
    def forward(ctx, hm, anchor, head, emb, labels, n_valid, model=None):
        """``n_valid``: host count of the non-ignored labels, or None (GPU: the normaliser is
        counted on the device — no host sync)."""
        c = head.cfg
        V, Vp, H, eps = c.vocab_size, c.vocab_padded, c.hidden_size, c.layer_norm_eps
        ctx.head, ctx.emb, ctx.model = head, emb, model
        ctx.native = use_native(hm)
        labels = labels.reshape(-1)
        if not ctx.native:
            ctx.save_for_backward(hm, labels)
            ctx.n_valid = n_valid
            with torch.no_grad():
                logits = mlm_head_ref(hm.float(), head.t_w.master, head.t_b.master, head.ln_g.master,
                                      head.ln_b.master, emb.word.master, head.dec_b.master, eps, V)
                return F.cross_entropy(logits, labels, ignore_index=-100, reduction="sum") / n_valid
        M = hm.shape[0]
        dev = hm.device
        pre = torch.empty((M, H), dtype=torch.bfloat16, device=dev)
        t = G.linear_fwd(hm, head.t_w.data, bias=head.t_b.master, act=G.ACT_GELU, aux=pre)
        t2 = torch.empty_like(t)
        mt = torch.empty(M, dtype=torch.float32, device=dev)
        rt = torch.empty_like(mt)
        C().layernorm_fwd(t, head.ln_g.master, head.ln_b.master, t2, mt, rt, eps)
        logits = G.linear_fwd(t2, emb.word.data, bias=head.dec_b.master)  # [M, Vp] (pad rows of E are zero)
        loss_rows = torch.empty(M, dtype=torch.float32, device=dev)
        dlogits = torch.empty_like(logits)
        labels = labels.long().contiguous()
        inv = None
        if n_valid is None:  # 1 / #valid labels on the device
            inv = torch.empty(1, dtype=torch.float32, device=dev)
            C().label_count_inv(labels, -100, inv)
        host_scale = 1.0 if inv is not None else 1.0 / n_valid
        C().softmax_xent(logits[:, :V], labels, None, loss_rows, dlogits[:, :V], host_scale, 0.0, -100, inv)
        ctx.save_for_backward(hm, pre, t, t2, mt, rt, dlogits)
        loss = torch.empty(1, dtype=torch.float32, device=dev)
        C().rows_sum_scaled(loss_rows, host_scale, inv, loss)
        return loss.view(())

    @staticmethod
    def backward(ctx, dloss):
        head, emb = ctx.head, ctx.emb
        c = head.cfg
        H, V, eps = c.hidden_size, c.vocab_size, c.layer_norm_eps
        if not ctx.native:
            hm, labels = ctx.saved_tensors
            prms = [head.t_w, head.t_b, head.ln_g, head.ln_b, emb.word, head.dec_b]

            def fn(h_, tw, tb, g, b, word, db):
                lg = mlm_head_ref(h_, tw, tb, g, b, word, db, eps, V)
                return F.cross_entropy(lg, labels, ignore_index=-100, reduction="sum") / ctx.n_valid

            grads = ref_grads(fn, [hm.float()] + [p.master for p in prms], dloss.float())
            for prm, g in zip(prms, grads[1:]):
                prm.grad.add_(g)
            if head.grad_hook is not None:
                head.grad_hook()
            return grads[0].to(hm.dtype), None, None, None, None, None, None
        hm, pre, t, t2, mt, rt, dlogits = ctx.saved_tensors
        # the incoming gradient is exactly 1 when a training step called loss.backward() (the model
        # flags it); otherwise it is applied on the device — never read back to the host
        if not getattr(ctx.model, "_unit_loss_grad", False):
            C().scale_bf16_dev(dlogits, dloss.detach().reshape(1).float().contiguous())
        M = hm.shape[0]
        _wgrad(dlogits, t2, emb.word.grad)  # tied decoder: dE += dlogits^T t2
        _bias_grad(dlogits, head.dec_b.grad)
        dt2 = _dgrad(dlogits, emb.word.data)
        dt = torch.empty_like(t)
        P_ = C().ln_bwd_rows(M, H)
        ws = torch.empty((P_, 2, H), dtype=torch.float32, device=hm.device)
        C().layernorm_bwd(dt2, t, mt, rt, head.ln_g.master, dt, None, 0.0, 0, ws)
        _ln_param_grads(ws, H, head.ln_g, head.ln_b)
        # t = gelu(pre): d(pre) = dt * gelu'(pre), one HIP elementwise pass (layer_ops.hip act_bwd, GELU code)
        dpre = torch.empty_like(dt)
        C().act_bwd(dt, pre, dpre, C().ACT_CODES["gelu"])
        _wgrad(dpre, hm, head.t_w.grad)
        _bias_grad(dpre, head.t_b.grad)
        dhm = _dgrad(dpre, head.t_w.data)
        if head.grad_hook is not None:
            head.grad_hook()
        return dhm, None, None, None, None, None, None


class _MaskedRowsFn(torch.autograd.Function):
    """hm[b P + i] = h[b S + pos[b, i]] (the MLM head's input rows) and its backward (a sum over duplicated
    positions), each ONE HIP launch (layernorm.hip mlm_gather / mlm_scatter)."""

    @staticmethod
    def forward(ctx, h, pos, S):
        out = torch.empty((pos.numel(), h.shape[1]), dtype=h.dtype, device=h.device)
        C().mlm_gather(h.contiguous(), pos, out, S)
        ctx.save_for_backward(pos)
        ctx.S, ctx.T = S, h.shape[0]
        return out

    @staticmethod
    def backward(ctx, dout):
        (pos,) = ctx.saved_tensors
        dh = torch.empty((ctx.T, dout.shape[1]), dtype=dout.dtype, device=dout.device)
        C().mlm_scatter(dout.contiguous(), pos, dh, ctx.S)
        return dh, None, None


def _gelu_grad(x):
    return 0.5 * (1.0 + torch.erf(x * 0.7071067811865476)) + x * 0.3989422804014327 * torch.exp(-0.5 * x * x)


# ====================================================================================== model
class BertForMaskedLM(Model):
    """``compute_loss(x, y)`` with ``x = {"input_ids": [B,S], "token_type_ids"?: [B,S],
    "lens"?: [B]}`` and ``y = {"positions": [B,P], "labels": [B,P] (-100 = padding),
    "num_masked"?: int}``."""

    def __init__(self, config: BertConfig | None = None, name=None, **kw):
        super().__init__(name=name or "bert_mlm", **kw)
        self.config = config or BertConfig()
        c = self.config
        self.embeddings = BertEmbeddings(c, name=self.name + "/embeddings")
        self.encoder = [BertLayer(c, i, name=f"{self.name}/encoder/layer_{i}") for i in range(c.num_hidden_layers)]
        self.head = BertMLMHead(c, name=self.name + "/cls/predictions")
        self._step = 0
        # the dropout hashes are seeded per replica: data-parallel ranks must not draw the same masks
        from ..ops.act import _process_rank

        self.dropout_seed = 1234 + 7919 * _process_rank()
        self.graph_capturable = False  # dropout hashes are seeded from a host step counter

    def sublayers(self):
        return [self.embeddings, *self.encoder, self.head]

    def build_model(self):
        if self.built:
            return
        for l in self.sublayers():
            l.ensure_built((self.config.hidden_size,))
        self.built = True

    def to_input(self, x):
        if isinstance(x, dict):
            return {k: (v if v is None else torch.as_tensor(np.asarray(v) if not torch.is_tensor(v) else v)
                        .to(self.device, non_blocking=True)) for k, v in x.items()}
        return {"input_ids": super().to_input(x)}

    def to_target(self, y):
        if isinstance(y, dict):
            return {k: (torch.as_tensor(v).to(self.device, non_blocking=True) if not isinstance(v, (int, float))
                        else v) for k, v in y.items()}
        return super().to_target(y)

    def encode(self, x, training=False):
        c = self.config
        ids = x["input_ids"]
        B, S = ids.shape
        types = x.get("token_type_ids")
        lens = x.get("lens")
        if lens is not None:
            lens = lens.to(torch.int32).contiguous()
        p_h = c.hidden_dropout_prob if training else 0.0
        p_a = c.attention_probs_dropout_prob if training else 0.0
        step = self._step
        anchor = self.embeddings.ln_g.data
        h = _EmbeddingsFn.apply(anchor, self.embeddings, ids.contiguous(), None if types is None else types.contiguous(),
                                S, p_h, _seed(self.dropout_seed, step, 0, 0))
        for i, layer in enumerate(self.encoder):
            seeds = tuple(_seed(self.dropout_seed, step, i + 1, k) for k in range(3))
            h = _BertLayerFn.apply(h, layer.ln1_g.data, layer, B, S, lens, p_h, p_a, seeds)
        return h  # [B*S, H]

    def compute_loss(self, x, y, training=True):
        if not isinstance(y, dict):
            raise ValueError("BertForMaskedLM expects y = {'positions': [B,P], 'labels': [B,P]}")
        h = self.encode(x, training)
        S = x["input_ids"].shape[1]
        pos = y["positions"].long()
        B, Pm = pos.shape
        if use_native(h):  # HIP row gather / scatter-sum (no arange, index_select, zero fill or index_add launches)
            hm = _MaskedRowsFn.apply(h, pos.contiguous(), S)
        else:
            flat = (pos + torch.arange(B, device=pos.device).view(B, 1) * S).reshape(-1)
            hm = h.index_select(0, flat)
        labels = y["labels"].reshape(-1).long()
        n_valid = y.get("num_masked")
        if n_valid is None and not use_native(hm):
            n_valid = int((labels != -100).sum().item())  # CPU tensors: no device sync involved
        if n_valid is not None:
            n_valid = max(1, int(n_valid))
        loss = _MLMHeadFn.apply(hm, self.head.ln_g.data, self.head, self.embeddings, labels, n_valid, self)
        if training:
            self._step += 1
        return loss

    def forward(self, x, training=False, logits=False):
        """Full-sequence MLM logits [B, S, V] (inference / evaluation).  GPU: the head is the
        training path's HIP kernels — transform GEMM with the GELU epilogue, LayerNorm, tied
        decoder GEMM with the bias epilogue, one HIP cast to fp32."""
        c = self.config
        B, S = x["input_ids"].shape
        with torch.no_grad():
            h = self.encode(x, False)
            hd = self.head
            if use_native(h):
                T_, H, V = h.shape[0], c.hidden_size, c.vocab_size
                pre = torch.empty((T_, H), dtype=torch.bfloat16, device=h.device)
                t = G.linear_fwd(h, hd.t_w.data, bias=hd.t_b.master, act=G.ACT_GELU, aux=pre)
                t2 = torch.empty_like(t)
                mt = torch.empty(T_, dtype=torch.float32, device=h.device)
                rt = torch.empty_like(mt)
                C().layernorm_fwd(t, hd.ln_g.master, hd.ln_b.master, t2, mt, rt, c.layer_norm_eps)
                lg16 = G.linear_fwd(t2, self.embeddings.word.data, bias=hd.dec_b.master)  # [T, Vp]
                lg = torch.empty((T_, lg16.shape[1]), dtype=torch.float32, device=h.device)
                C().cast_bf16_f32(lg16, lg)
                return lg.view(B, S, -1)[..., :V]
            lg = mlm_head_ref(h.float(), hd.t_w.master, hd.t_b.master, hd.ln_g.master, hd.ln_b.master,
                              self.embeddings.word.master, hd.dec_b.master, c.layer_norm_eps, c.vocab_size)
        return lg.view(B, S, -1)

    def get_config(self):
        return {"name": self.name, "config": asdict(self.config)}

    @classmethod
    def from_config(cls, cfg):
        return cls(BertConfig(**cfg["config"]), name=cfg.get("name"))

    def summary_rows(self):
        return [(f"{l.name} ({type(l).__name__})", "", l.count_params()) for l in self.sublayers()]


def bert_base_mlm(**kw) -> BertForMaskedLM:
    return BertForMaskedLM(BertConfig.base(**kw))
