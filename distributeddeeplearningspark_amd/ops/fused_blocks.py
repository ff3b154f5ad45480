"""Fused ResNet bottleneck (GPU): the whole conv-BN-ReLU x3 + shortcut block is ONE
autograd node whose backward is scheduled by hand.

What the fusion buys over composing per-op autograd nodes:
  * the block-input gradient ``dX = dgrad(conv1) + dShortcut`` is produced by the
    conv1 data-gradient GEMM epilogue (residual add), instead of a separate add kernel;
  * every BN uses the statistics the producing conv's epilogue accumulated;
  * the BN backward ReLU masks are recomputed from the conv outputs (mode 2) except
    where a residual enters (mode 1), so no extra activation tensor is read;
  * all workspaces come from the per-step statistics pool;
  * parameter-gradient hooks (for the overlapped RCCL all-reduce) fire per layer in
    backward order as soon as each layer's gradients are final.
Reference semantics are unchanged: ``relu(bn3(conv3(relu(bn2(conv2(relu(bn1(conv1 x))))))) + sc(x))``.
"""
from __future__ import annotations

import weakref

import torch

from . import conv as CV
from . import determinism as _det
from . import gemm as G
from . import zpad as ZP
from ._native import C
from .norm import new_stats_workspace, partials_workspace
from .streams import on_grad_stream


class _ConvBNState:
    """Per-(conv,BN) forward results needed by the backward.  ``pre_reduced``: the BN-backward
    partial sums [32, 2, C] already accumulated by the producer of this BN's output gradient
    (the next block's conv1 data-gradient epilogue), so ``bn_backward`` skips its reduce sweep."""

    __slots__ = ("g", "yc", "y", "mean", "invstd", "scale", "shift", "mode", "mask", "pre_reduced", "__weakref__")

    def __init__(self):
        self.pre_reduced = None


# Block outputs -> the (ConvBN unit, state) of the BN that produced them (weak references only): the
# next bottleneck looks its input up here so that, in backward, its conv1 data-gradient (which
# produces THIS BN's output gradient) can also accumulate this BN's backward partial sums.
_PRODUCERS: dict = {}


def _register_output(y, unit, st):
    _PRODUCERS[y.data_ptr()] = (weakref.ref(y), unit, weakref.ref(st))
    if len(_PRODUCERS) > 4096:  # stale entries of freed tensors
        for k in [k for k, v in _PRODUCERS.items() if v[0]() is None]:
            del _PRODUCERS[k]


def _producer_of(x):
    e = _PRODUCERS.get(x.data_ptr())
    if e is None or e[0]() is not x:
        return None
    st = e[2]()
    return None if st is None else (e[1], st)


def _bn_forward(layer_bn, yc, stats, resid, relu, training, mask=None, apply=True, res_affine=None):
    """Finalize the fused statistics into scale/shift (+ running stats) and, with ``apply``, write
    ``relu(yc * scale + shift + resid)``; ``res_affine = (scale_r, shift_r)`` normalises a pre-BN
    residual on the fly (the downsample shortcut's BN rides in its consumer's apply sweep)."""
    Cc = yc.shape[-1]
    M = yc.numel() // Cc
    dev = yc.device
    bn = layer_bn
    gamma = None if bn.gamma is None else bn.gamma.master
    beta = None if bn.beta is None else bn.beta.master
    rm, rv = bn._states["moving_mean"], bn._states["moving_variance"]
    # one allocation for the four per-channel vectors (host cost per BN: VGG-16 runs launch-bound)
    scale, shift, mean, invstd = torch.empty(4, Cc, dtype=torch.float32, device=dev).unbind(0)
    if stats is None:  # deterministic mode: no fused (atomic) statistics; fixed-order partial rows instead
        stats = partials_workspace(M, Cc, dev)
        C().bn_stats(yc, stats, Cc)
    C().bn_finalize(stats, M, Cc, gamma, beta, bn.epsilon, 1.0 - bn.momentum, rm, rv, mean, invstd, scale, shift)
    if not apply:
        return None, mean, invstd, scale, shift
    y = torch.empty_like(yc)
    rs, rt = res_affine if res_affine is not None else (None, None)
    C().bn_apply(yc, scale, shift, resid, y, Cc, relu, mask, rs, rt)
    return y, mean, invstd, scale, shift


def convbn_forward(unit, x, resid=None, relu=True, apply=True, res_affine=None):
    """conv (fused statistics) + BN (+resid)(+relu) for a ``models.resnet.ConvBN`` unit.
    ``apply=False``: statistics and scale/shift only (``st.y`` is None: the consumer applies them)."""
    conv, bn = unit.conv, unit.bn
    N, H, W, Ci = x.shape
    kh, kw = conv.kernel_size
    p = conv.padding if isinstance(conv.padding, tuple) else (kh // 2, kw // 2)
    g = CV.geometry(N, H, W, Ci, conv.filters, kh, kw, conv.strides, p, conv.dilation_rate)
    stats = new_stats_workspace(conv.filters, x.device)
    yc = CV.conv_fwd_native(x, conv.kernel.data, g, stats=stats)
    st = _ConvBNState()
    st.g, st.yc = g, yc
    # ReLU after a residual add: the backward mask cannot be recomputed from yc alone, so the
    # apply pass stores it as bits (mode 3) instead of the backward re-reading the bf16 output
    bits = relu and resid is not None
    st.mask = torch.empty(-(-yc.numel() // 32) * 4, dtype=torch.uint8, device=yc.device) if bits else None
    st.y, st.mean, st.invstd, st.scale, st.shift = _bn_forward(bn, yc, stats, resid, relu, True, st.mask, apply,
                                                               res_affine)
    st.mode = 0 if not relu else (2 if resid is None else (3 if bits else 1))
    return st


def bn_backward(unit, st, dy, want_dres, red2=None, dy_mask=None, reduced=None):
    """BN backward of ``st`` for output gradient ``dy``: (dx, dres or None).

    ``red2 = (x2, mean2, ws2)``: the dx sweep also writes the reduce partials of a second BN fed by the
    masked gradient (``bn_bwd_dx_red``; the ResNet downsample BN).  ``dy_mask``: the gradient this BN
    sees is ``dy`` under that ReLU bit mask (mode 3), i.e. the masked gradient is never materialised;
    ``reduced``: the partial-sum workspace already holds this BN's reduce (the red2 of the producer)."""
    bn = unit.bn
    Cc = st.yc.shape[-1]
    M = st.yc.numel() // Cc
    mode = st.mode
    y = st.y if st.mode == 1 else (st.mask if st.mode == 3 else None)
    if dy_mask is not None:
        if st.mode != 0:
            raise ValueError("bn_backward: dy_mask applies to a BN without its own ReLU")
        mode, y = 3, dy_mask
    pre, st.pre_reduced = st.pre_reduced, None
    if reduced is not None:
        ws = reduced
    elif pre is not None and _same_tensor(pre[1], dy):
        # partial sums already accumulated by dy's producer (no reduce sweep) — valid only when dy IS the
        # gradient that producer reduced: a second consumer of this BN's output makes autograd sum the
        # gradients into a new tensor, and then the sweep runs on the sum
        ws = pre[0]
    else:
        ws = partials_workspace(M, Cc, dy.device)
        C().bn_bwd_reduce(dy, st.yc, y, st.scale, st.shift, st.mean, ws, Cc, mode)
    coef = torch.empty(3 * Cc, dtype=torch.float32, device=dy.device)
    C().bn_bwd_finalize(ws, M, Cc, None if bn.gamma is None else bn.gamma.master, st.mean, st.invstd,
                        None if bn.gamma is None else bn.gamma.grad, None if bn.beta is None else bn.beta.grad, coef)
    dyc = torch.empty_like(dy)
    dres = torch.empty_like(dy) if want_dres else None
    if red2 is not None:
        if dres is not None:
            raise ValueError("bn_backward: red2 replaces dres")
        C().bn_bwd_dx_red(dy, st.yc, y, st.scale, st.shift, coef, dyc, Cc, mode, red2[0], red2[1], red2[2])
    else:
        C().bn_bwd_dx(dy, st.yc, y, st.scale, st.shift, coef, dyc, dres, Cc, mode)
    if bn.grad_hook is not None:
        bn.grad_hook()
    return dyc, dres


def conv_backward(unit, st, dyc, x, need_dx, resid=None, resid_mask=None, bnr=None, rsub=None):
    conv = unit.conv
    # the weight gradient only feeds the optimizer / all-reduce: it runs on the side stream
    # (ops/streams.py) beside the data-gradient and BatchNorm sweeps of the layers below
    # (every tensor the side-stream kernel reads is recorded on that stream: the main stream may
    # drop them before the side stream has run)
    with on_grad_stream(dyc.device, dyc, x, default=False):
        CV.conv_wgrad_native(dyc, x, st.g, conv.kernel.grad)
    dx = None
    if need_dx:
        dx = CV.conv_dgrad_native(dyc, conv.kernel.data, st.g, resid=resid, resid_mask=resid_mask, bnr=bnr, rsub=rsub)
    # the hook comes after the last read of the weights: on one GPU it may start the optimizer on this bucket
    # (parallel/ddp.py DataParallel.solo), which rewrites them
    if conv.grad_hook is not None:
        conv.grad_hook()
    return dx


class _BottleneckFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, block):
        ctx.prev = _producer_of(x) if _FUSE_BNR else None  # the BN whose output is this block's input
        x = x.contiguous()
        # the downsample BN is not applied on its own: its scale/shift normalise the shortcut inside
        # the block-output apply sweep (one write + one read of the shortcut tensor saved)
        s_down = convbn_forward(block.down, x, relu=False, apply=False) if block.down is not None else None
        sc = s_down.yc if s_down is not None else x
        s1 = convbn_forward(block.c1, x, relu=True)
        s2 = convbn_forward(block.c2, s1.y, relu=True)
        s3 = convbn_forward(block.c3, s2.y, resid=sc, relu=True,
                            res_affine=None if s_down is None else (s_down.scale, s_down.shift))
        ctx.block, ctx.states = block, (s_down, s1, s2, s3)
        ctx.save_for_backward(x)
        ctx.needs_dx = ctx.needs_input_grad[0]
        _register_output(s3.y, block.c3, s3)
        return s3.y

    @staticmethod
    def backward(ctx, dout):
        (x,) = ctx.saved_tensors
        b = ctx.block
        s_down, s1, s2, s3 = ctx.states
        dout = dout.contiguous()
        # identity shortcut: its gradient is dout masked by the block-output ReLU; instead of the BN
        # backward writing it out, conv1's data-gradient epilogue adds dout under the bit mask
        masked_sc = s_down is None and s3.mode == 3 and s1.g.is_pointwise
        # downsample shortcut: its BN's input gradient is dout under bn3's ReLU mask.  bn3's dx sweep also
        # writes that BN's reduce partials (it reads dout and the mask anyway; + a read of the shortcut's
        # pre-BN tensor), and the shortcut BN's dx sweep re-applies the mask to dout — so the masked
        # gradient is never written, and the shortcut BN runs no reduce sweep
        fuse_down = _FUSE_DOWN and s_down is not None and s3.mode == 3 and s_down.mode == 0
        ws_d = None
        if fuse_down:
            Cd = s_down.yc.shape[-1]
            ws_d = partials_workspace(s_down.yc.numel() // Cd, Cd, dout.device)
            d3c, dsc = bn_backward(b.c3, s3, dout, False, red2=(s_down.yc, s_down.mean, ws_d))
        else:
            d3c, dsc = bn_backward(b.c3, s3, dout, want_dres=not masked_sc)
        # the data-gradients of conv3 and conv2 produce bn2's / bn1's output gradients: their epilogues also
        # accumulate those BNs' backward partial sums (ReLU mask recomputed from yc), so bn_backward skips the
        # reduce sweep wherever the kernel that ran could take it (bnr["done"])
        bnr2 = _bnr_mode2(s2, dout.device)
        d2 = conv_backward(b.c3, s3, d3c, s2.y, True, bnr=bnr2)
        _take_reduced(s2, bnr2, d2)
        d2c, _ = bn_backward(b.c2, s2, d2, False)
        bnr1 = _bnr_mode2(s1, dout.device)
        d1 = conv_backward(b.c2, s2, d2c, s1.y, True, bnr=bnr1)
        _take_reduced(s1, bnr1, d1)
        d1c, _ = bn_backward(b.c1, s1, d1, False)
        rsub = None
        if s_down is not None:
            if fuse_down:
                ddc, _ = bn_backward(b.down, s_down, dout, False, dy_mask=s3.mask, reduced=ws_d)
            else:
                ddc, _ = bn_backward(b.down, s_down, dsc, False)
            gd = s_down.g
            if (_HALF_RES_SC and ctx.needs_dx and s1.g.is_pointwise and gd.KH == 1 and gd.KW == 1
                    and (gd.sh, gd.sw) == (2, 2) and (gd.ph, gd.pw) == (0, 0)):
                # stride-2 1x1 shortcut: its data-gradient stays at half resolution ([N, H/2, W/2, Cin], a plain
                # GEMM) and conv1's dgrad epilogue adds it at the even pixels — instead of a scatter GEMM that
                # writes a full-resolution tensor of 3/4 zeros which that epilogue then reads back
                wd = b.down.conv.kernel.data
                dsc = G.linear_dgrad(ddc.view(gd.M, gd.Co), wd.view(gd.Co, gd.Ci))
                rsub = (gd.H, gd.W)
                conv_backward(b.down, s_down, ddc, x, False)  # weight gradient + hook, after the last weight read
            else:
                dsc = conv_backward(b.down, s_down, ddc, x, ctx.needs_dx)
        # dX = dgrad(conv1) + dShortcut: the residual add rides in the conv1 dgrad epilogue, and so do the
        # backward partial sums of the BN that produced X (previous block's bn3, mode 3) when that GEMM
        # runs on the streaming kernel — that BN's backward then skips its reduce sweep over dX and yc
        bnr = None
        if ctx.needs_dx and ctx.prev is not None and ctx.prev[1].mode == 3 and not _det.enabled():
            pst = ctx.prev[1]
            bnr = {"x": pst.yc, "mask": pst.mask, "mean": pst.mean,
                   "ws": new_stats_workspace(pst.yc.shape[-1], dout.device)}
        if _TEST_MUTATION is not None and _TEST_MUTATION[0] == "drop_shortcut" and _TEST_MUTATION[1] in (None, b.name):
            # test-only fault (tests/test_gpu_determinism.py): the block's input gradient loses its shortcut term
            masked_sc, dsc, rsub = False, None, None
        if masked_sc:
            dx = conv_backward(b.c1, s1, d1c, x, ctx.needs_dx, resid=dout, resid_mask=s3.mask, bnr=bnr)
        else:
            dx = conv_backward(b.c1, s1, d1c, x, ctx.needs_dx, resid=dsc, bnr=bnr, rsub=rsub)
        if bnr is not None and bnr.get("done"):
            ctx.prev[1].pre_reduced = (bnr["ws"], dx)
        ctx.states = ctx.prev = None
        return dx, None, None



_FUSE_BNR = True
# test-only fault injection for the discriminating gradient checks: ("drop_shortcut", block name or None)
_TEST_MUTATION = None
# bn1 / bn2 of every bottleneck: reduce fused into the conv2 / conv3 data-gradient epilogues
_FUSE_BNR_INNER = True
_HALF_RES_SC = True
# downsample BN backward fed by bn3's dx sweep (bn_bwd_dx_red): no masked-gradient tensor, no reduce sweep
_FUSE_DOWN = True
# stem: BN backward through the max pool without materialising the pool's gradient (pool3s2_bn_bwd)
_FUSE_STEM_BWD = True
_STEM_PARTIALS = 2048  # workgroups (= partial rows) of its reduce


def _bnr_mode2(st, device):
    """BN-backward reduce request for a ReLU BN without residual (mode 2) — see ``gemm.linear_dgrad``."""
    if not _FUSE_BNR_INNER or st.mode != 2 or _det.enabled():
        return None
    return {"x": st.yc, "scale": st.scale, "shift": st.shift, "mean": st.mean,
            "ws": new_stats_workspace(st.yc.shape[-1], device)}


def _take_reduced(st, bnr, d):
    if bnr is not None and bnr.get("done"):
        st.pre_reduced = (bnr["ws"], d)


def _same_tensor(a, b) -> bool:
    """b is the very gradient tensor a (same storage, shape and version), not a sum formed from it."""
    return (a.data_ptr() == b.data_ptr() and a.shape == b.shape and a.stride() == b.stride()
            and a._version == b._version)


def bottleneck(block, x, anchor):
    """``anchor``: any parameter view requiring grad (makes the node part of the graph)."""
    return _BottleneckFn.apply(x, anchor, block)


def convbn_relu(unit, x, anchor, relu=True):
    """Single fused conv+BN(+ReLU) unit as one autograd node (the ResNet stem)."""
    if not x.requires_grad and _stem_s2d_ok(unit.conv, x.shape[-1]):
        return _StemS2DFn.apply(x, anchor, unit, relu)
    return _ConvBNFn.apply(x, anchor, unit, relu)


_STEM_S2D = True  # space-to-depth stem (tests switch it off to compare with the plain 7x7 conv)
_STEM_POOL = True  # stem conv + BN + ReLU + max pool as one node


def _stem_s2d_ok(conv, Ci) -> bool:
    """7x7 / stride 2 / pad 3 stem on <= 4 channels: run as a 4x4 stride-1 conv after a
    block-2 space-to-depth (12 of 16 channels used instead of 3 of 8, K = 256 instead of 392)."""
    return (_STEM_S2D and Ci <= 4 and tuple(conv.kernel_size) == (7, 7)
            and tuple(conv.strides) == (2, 2) and tuple(conv.dilation_rate) == (1, 1)
            and (conv.padding == (3, 3) or conv.padding == 3 or conv.padding == "same"))


def _s2d_weight(w):
    """[Co, 7, 7, C] -> [Co, 4, 4, 16]: W'[A][B][(2a+b)C + ch] = W[2A+a][2B+b][ch] (zero past 7)."""
    Co, _, _, Cc = w.shape
    w8 = torch.nn.functional.pad(w, (0, 0, 0, 1, 0, 1))  # [Co, 8, 8, C]
    w4 = w8.view(Co, 4, 2, 4, 2, Cc).permute(0, 1, 3, 2, 4, 5).reshape(Co, 4, 4, 4 * Cc)
    return torch.nn.functional.pad(w4, (0, 16 - 4 * Cc)).contiguous()


def _s2d_weight_grad(g4, Cc):
    """Inverse of _s2d_weight for gradients: [Co, 4, 4, 16] -> [Co, 7, 7, C]."""
    Co = g4.shape[0]
    g = g4[..., : 4 * Cc].reshape(Co, 4, 4, 2, 2, Cc).permute(0, 1, 3, 2, 4, 5).reshape(Co, 8, 8, Cc)
    return g[:, :7, :7, :]


_S2D_TABLES: dict = {}


def _s2d_table(t):
    """(int32 [Co, 4, 4, 16] table, extent): entry i of the space-to-depth filter is element table[i] of
    ``t``'s storage from ``t.data_ptr()`` (its own strides: the arena's padded views work), -1 = zero.
    The same table gathers the bf16 filter (forward) and scatters the fp32 gradient back (backward)."""
    key = (tuple(t.shape), tuple(t.stride()), str(t.device))
    hit = _S2D_TABLES.get(key)
    if hit is None:
        offs = torch.zeros((), dtype=torch.int64)
        for d, (n, st) in enumerate(zip(t.shape, t.stride())):
            offs = offs.unsqueeze(-1) + torch.arange(n, dtype=torch.int64) * st
        Co, _, _, Cc = t.shape
        o8 = torch.nn.functional.pad(offs, (0, 0, 0, 1, 0, 1), value=-1)
        o4 = o8.view(Co, 4, 2, 4, 2, Cc).permute(0, 1, 3, 2, 4, 5).reshape(Co, 4, 4, 4 * Cc)
        tab = torch.nn.functional.pad(o4, (0, 16 - 4 * Cc), value=-1).contiguous()
        hit = _S2D_TABLES[key] = (tab.to(torch.int32).to(t.device), int(offs.max()) + 1)
    return hit


def _s2d_weight_dev(w):
    """``_s2d_weight`` as one table-driven HIP gather (no pad / permute / copy kernels per step)."""
    if not (w.is_cuda and w.dtype == torch.bfloat16):
        return _s2d_weight(w)
    tab, ext = _s2d_table(w)
    out = torch.empty(tab.shape, dtype=w.dtype, device=w.device)
    C().gather_bf16(w, tab, out, ext)
    return out


def _s2d_weight_grad_into(conv, g, dyc, xs, Cc):
    """Stem weight gradient: the 4x4 conv's gradient into a zeroed scratch, scattered (added) into the
    7x7 filter's gradient by the gather table's adjoint — HIP launches only."""
    gw = conv.kernel.grad
    tmp = torch.empty((g.Co, 4, 4, 16), dtype=torch.float32, device=dyc.device)
    if not gw.is_cuda:
        tmp.zero_()
        CV.conv_wgrad_native(dyc, xs, g, tmp)
        gw.add_(_s2d_weight_grad(tmp, Cc))
        return
    C().zero_ranges([tmp])
    CV.conv_wgrad_native(dyc, xs, g, tmp)
    tab, ext = _s2d_table(gw)
    C().scatter_add_f32(tmp, tab, gw, ext)


class _StemPoolFn(torch.autograd.Function):
    """ResNet stem conv (7x7 s2 p3 through space-to-depth) + BN + ReLU + 3x3/2 max pool as ONE node:
    the BN affine and ReLU are applied by the pool as it loads the conv output (maxpool_fwd with
    scale/shift), so the stem's BN-apply sweep — a write and a re-read of the largest activation of
    the network (batch 256: 411 MB each way) — is gone.  Backward: pool gather -> BN backward (ReLU
    mask recomputed from the conv output, mode 2) -> weight gradient, as before."""

    @staticmethod
    def forward(ctx, x, anchor, unit, k, s, p):
        x = x.contiguous()
        N, H, W, Cc = x.shape
        conv = unit.conv
        Ho, Wo = (H + 6 + 1) // 2, (W + 6 + 1) // 2
        xs = torch.empty((N, Ho, Wo, 16), dtype=x.dtype, device=x.device)
        C().s2d_pad(x, xs, 3)
        w4 = _s2d_weight_dev(conv.kernel.data.detach())
        g = CV.geometry(N, Ho, Wo, 16, conv.filters, 4, 4, (1, 1), (0, 0), (1, 1))
        stats = new_stats_workspace(conv.filters, x.device)
        yc = CV.conv_fwd_native(xs, w4, g, stats=stats)
        st = _ConvBNState()
        st.g, st.yc = g, yc
        st.y, st.mean, st.invstd, st.scale, st.shift = _bn_forward(unit.bn, yc, stats, None, True, True, apply=False)
        st.mode = 2
        _, Hc, Wc, Co = yc.shape
        Hp, Wp = (Hc + 2 * p - k) // s + 1, (Wc + 2 * p - k) // s + 1
        y = torch.empty((N, Hp, Wp, Co), dtype=yc.dtype, device=yc.device)
        am = torch.empty((N, Hp, Wp, Co), dtype=torch.uint8, device=yc.device)
        C().maxpool_fwd(yc, y, am, k, k, s, s, p, p, st.scale, st.shift)
        ctx.unit, ctx.st, ctx.cc, ctx.pool = unit, st, Cc, (k, s, p)
        ctx.save_for_backward(xs, am)
        return y

    @staticmethod
    def backward(ctx, dy):
        xs, am = ctx.saved_tensors
        unit, st = ctx.unit, ctx.st
        k, s, p = ctx.pool
        dy = dy.contiguous()
        N, H, W, Co = st.yc.shape
        if _FUSE_STEM_BWD and (k, s, p) == (3, 2, 1) and C().pool3s2_bn_bwd_ok(N, H, W, Co, dy.shape[1], dy.shape[2], 3):
            # the BN output gradient (the pool's gather) is recomputed from dy + argmax by the reduce and the dx
            # sweeps instead of being written (411 MB at batch 256) and read back by both
            bn = unit.bn
            M = N * H * W
            ws = torch.empty((_STEM_PARTIALS, 2, Co), dtype=torch.float32, device=dy.device)  # one row per workgroup
            C().pool3s2_bn_bwd(dy, am, st.yc, st.scale, st.shift, st.mean, ws, None)
            coef = torch.empty(3 * Co, dtype=torch.float32, device=dy.device)
            C().bn_bwd_finalize(ws, M, Co, None if bn.gamma is None else bn.gamma.master, st.mean, st.invstd,
                                None if bn.gamma is None else bn.gamma.grad, None if bn.beta is None else bn.beta.grad,
                                coef)
            dyc = torch.empty_like(st.yc)
            C().pool3s2_bn_bwd(dy, am, st.yc, st.scale, st.shift, st.mean, coef, dyc)
            if bn.grad_hook is not None:
                bn.grad_hook()
        else:
            d = torch.empty_like(st.yc)
            C().maxpool_bwd(dy, am, d, k, k, s, s, p, p)
            dyc, _ = bn_backward(unit, st, d, False)
        conv = unit.conv
        g = st.g
        with on_grad_stream(dy.device, dyc, xs, default=False):
            _s2d_weight_grad_into(conv, g, dyc, xs, ctx.cc)
        if conv.grad_hook is not None:
            conv.grad_hook()
        ctx.st = None
        return None, None, None, None, None, None  # the stem input is data: no gradient


def stem_pool(unit, x, anchor, k=3, s=2, p=1):
    """Stem conv+BN+ReLU followed by a k x k / s max pool, fused when the space-to-depth stem applies
    (``_STEM_POOL = False`` keeps the separate apply + pool); returns None when not applicable."""
    if (not _STEM_POOL or x.requires_grad or not _stem_s2d_ok(unit.conv, x.shape[-1])
            or unit.conv.filters % 8):
        return None
    return _StemPoolFn.apply(x, anchor, unit, k, s, p)


class _StemS2DFn(torch.autograd.Function):
    """ResNet stem conv (7x7 s2 p3, 3 channels) + BN (+ReLU) through space-to-depth."""

    @staticmethod
    def forward(ctx, x, anchor, unit, relu):
        x = x.contiguous()
        N, H, W, Cc = x.shape
        conv = unit.conv
        Ho, Wo = (H + 6 + 1) // 2, (W + 6 + 1) // 2
        xs = torch.empty((N, Ho, Wo, 16), dtype=x.dtype, device=x.device)
        C().s2d_pad(x, xs, 3)
        w4 = _s2d_weight_dev(conv.kernel.data.detach())
        g = CV.geometry(N, Ho, Wo, 16, conv.filters, 4, 4, (1, 1), (0, 0), (1, 1))
        stats = new_stats_workspace(conv.filters, x.device)
        yc = CV.conv_fwd_native(xs, w4, g, stats=stats)
        st = _ConvBNState()
        st.g, st.yc = g, yc
        st.y, st.mean, st.invstd, st.scale, st.shift = _bn_forward(unit.bn, yc, stats, None, relu, True)
        st.mode = 2 if relu else 0
        ctx.unit, ctx.st, ctx.cc = unit, st, Cc
        ctx.save_for_backward(xs)
        return st.y

    @staticmethod
    def backward(ctx, dy):
        (xs,) = ctx.saved_tensors
        unit, st = ctx.unit, ctx.st
        dyc, _ = bn_backward(unit, st, dy.contiguous(), False)
        conv = unit.conv
        g = st.g
        with on_grad_stream(dy.device, dyc, xs, default=False):
            _s2d_weight_grad_into(conv, g, dyc, xs, ctx.cc)
        if conv.grad_hook is not None:
            conv.grad_hook()
        ctx.st = None
        return None, None, None, None  # the stem input is data: no gradient


def _seq_conv_forward(ctx, x, unit):
    """Conv half of a Sequential conv -> BN node (``_ConvBNFn`` / ``_ConvBNPoolFn``): the conv output with
    its BN statistics fused into the epilogue; records on ``ctx`` what the backward needs."""
    # a conv -> BN -> ReLU chain (VGG): this conv's data-gradient epilogue accumulates the backward
    # partial sums of the BN that produced x (mode 2), whose backward then skips its reduce sweep
    ctx.prev = _producer_of(x) if _FUSE_BNR else None
    x = x.contiguous()
    Ci = x.shape[-1]
    ctx.ci = Ci
    kp = unit.conv.kernel
    if Ci % 8:  # stem: pad 3 -> 8 channels (16-B vectors); the arena keeps the filter padded (params.py)
        cp = -(-Ci // 8) * 8
        x = ZP.padded(x, cp)
        w = kp.pdata if kp.pshape[1:] == (*kp.shape[1:3], cp) and kp.pshape[0] == kp.shape[0] \
            else torch.nn.functional.pad(kp.data.detach(), (0, cp - Ci))
    else:
        w = kp.data
    conv = unit.conv
    N, H, W, Cp = x.shape
    kh, kw = conv.kernel_size
    p = conv.padding if isinstance(conv.padding, tuple) else (kh // 2, kw // 2)
    g = CV.geometry(N, H, W, Cp, conv.filters, kh, kw, conv.strides, p, conv.dilation_rate)
    stats = new_stats_workspace(conv.filters, x.device)
    yc = CV.conv_fwd_native(x, w, g, stats=stats)
    st = _ConvBNState()
    st.g, st.yc = g, yc
    ctx.unit, ctx.st, ctx.w, ctx.x = unit, st, w, x
    ctx.needs_dx = ctx.needs_input_grad[0]
    return st, stats


def _seq_conv_backward(ctx, dyc):
    """Weight gradient (side stream) and data gradient of the conv half, given the conv output's gradient."""
    unit, x = ctx.unit, ctx.x
    conv = unit.conv
    g = ctx.st.g
    with on_grad_stream(dyc.device, dyc, x, default=False):
        if g.Ci != ctx.ci and ctx.w is not conv.kernel.pdata:
            tmp = torch.zeros((g.Co, g.KH, g.KW, g.Ci), dtype=torch.float32, device=dyc.device)
            CV.conv_wgrad_native(dyc, x, g, tmp)
            conv.kernel.grad.add_(tmp[..., : ctx.ci])
        else:  # padded storage: it takes the zero-padded channels' (zero) gradients as is
            CV.conv_wgrad_native(dyc, x, g, conv.kernel.pgrad if ctx.w is conv.kernel.pdata else conv.kernel.grad)
    dx = None
    if ctx.needs_dx:
        bnr = None if ctx.prev is None else _bnr_mode2(ctx.prev[1], dyc.device)
        dx = CV.conv_dgrad_native(dyc, ctx.w, g, bnr=bnr)
        if bnr is not None:
            _take_reduced(ctx.prev[1], bnr, dx)
        dx = ZP.logical(dx, ctx.ci)
    if conv.grad_hook is not None:  # after the last read of the weights (see conv_backward)
        conv.grad_hook()
    ctx.st = ctx.prev = ctx.x = None
    return dx


class _ConvBNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, unit, relu):
        st, stats = _seq_conv_forward(ctx, x, unit)
        st.y, st.mean, st.invstd, st.scale, st.shift = _bn_forward(unit.bn, st.yc, stats, None, relu, True)
        st.mode = 2 if relu else 0
        _register_output(st.y, unit, st)
        return st.y

    @staticmethod
    def backward(ctx, dy):
        dyc, _ = bn_backward(ctx.unit, ctx.st, dy.contiguous(), False)
        return _seq_conv_backward(ctx, dyc), None, None, None


_SEQ_POOL = True  # Sequential conv -> BN -> ReLU -> 2x2 / 2 max pool as one node (tests compare with False)


class _ConvBNPoolFn(torch.autograd.Function):
    """VGG block tail conv -> BN -> ReLU -> 2x2 / stride-2 max pool as ONE node: the pool applies the BN
    affine + ReLU as it loads the conv output (no BN-apply sweep, the full-resolution activation is never
    written); backward: the BN's output gradient is the pool's scatter of the pooled gradient by the argmax
    bytes, recomputed inside the reduce and dx sweeps (``pool_bn_bwd``, k = 2) instead of written by a pool
    backward and read twice."""

    @staticmethod
    def forward(ctx, x, anchor, unit):
        st, stats = _seq_conv_forward(ctx, x, unit)
        st.y, st.mean, st.invstd, st.scale, st.shift = _bn_forward(unit.bn, st.yc, stats, None, True, True,
                                                                    apply=False)
        st.mode = 2
        N, Hc, Wc, Co = st.yc.shape
        y = torch.empty((N, Hc // 2, Wc // 2, Co), dtype=st.yc.dtype, device=st.yc.device)
        ctx.am = torch.empty(y.shape, dtype=torch.uint8, device=y.device)
        C().maxpool_fwd(st.yc, y, ctx.am, 2, 2, 2, 2, 0, 0, st.scale, st.shift)
        return y

    @staticmethod
    def backward(ctx, dy):
        st, bn = ctx.st, ctx.unit.bn
        dy = dy.contiguous()
        N, H, W, Co = st.yc.shape
        M = N * H * W
        # one partial row per workgroup, each workgroup one pass over its 256 / (C / 8) rows of 2x2 blocks
        rows = -(-(N * (H // 2) * (W // 2)) // max(1, 256 // (Co // 8)))
        ws = torch.empty((min(_STEM_PARTIALS, rows), 2, Co), dtype=torch.float32, device=dy.device)
        C().pool3s2_bn_bwd(dy, ctx.am, st.yc, st.scale, st.shift, st.mean, ws, None, 2)
        coef = torch.empty(3 * Co, dtype=torch.float32, device=dy.device)
        C().bn_bwd_finalize(ws, M, Co, bn.gamma.master, st.mean, st.invstd, bn.gamma.grad, bn.beta.grad, coef)
        dyc = torch.empty_like(st.yc)
        C().pool3s2_bn_bwd(dy, ctx.am, st.yc, st.scale, st.shift, st.mean, coef, dyc, 2)
        if bn.grad_hook is not None:
            bn.grad_hook()
        ctx.am = None
        return _seq_conv_backward(ctx, dyc), None, None


def convbn_relu_pool(unit, x, anchor):
    """Sequential conv -> BN -> ReLU -> MaxPooling2D(2, 2) as one node, or None when it does not apply."""
    conv = unit.conv
    if not _SEQ_POOL or conv.filters % 8 or conv.filters > 2048 or tuple(conv.strides) != (1, 1):
        return None
    if not (x.is_cuda and x.dtype == torch.bfloat16) or x.shape[1] % 2 or x.shape[2] % 2:
        return None
    return _ConvBNPoolFn.apply(x, anchor, unit)


_ = G
