"""NHWC 2-D convolution on MFMA implicit GEMM.

Layouts: activations ``[N, H, W, C]`` (bf16 on GPU), weights ``[Co, KH, KW, Ci]``
(K-contiguous for the forward GEMM).  Parameter gradients are accumulated out of
band into fp32 gradient-arena views (``gw``, ``gb``), so autograd only tracks
activations and the data-parallel engine is told when each gradient is final.

Decomposition (``ConvGeometry``):
  forward  : M = N*Ho*Wo pixels, N = Co, K = taps*Ci.  1x1/stride-1 is a plain GEMM;
             Ci % 64 == 0 gathers A through a tap table (implicit GEMM, zero padding
             handled in the loader); other Ci (stem, MNIST) use an im2col pass.
  dgrad    : the transposed convolution as implicit GEMM over dY with a flipped tap
             table; stride s is split into s*s parity classes, each a stride-1 problem
             whose rows scatter to a strided grid (OutMap) — no col2im, no atomics.
  wgrad    : M = Co, N = taps*Ci, K = N*Ho*Wo with split-K and fp32 accumulation;
             A = dY read row-contiguous, B = X gathered per tap.
"""
from __future__ import annotations

import math
from functools import lru_cache

import torch
import torch.nn.functional as F

from . import determinism as _det
from . import derived
from . import gemm as G
from . import zpad as ZP
from ._native import C, use_native
from ._ref import accumulate, ref_grads
from .streams import on_grad_stream


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


class ConvGeometry:
    def __init__(self, N, H, W, Ci, Co, KH, KW, stride, pad, dil):
        self.N, self.H, self.W, self.Ci, self.Co, self.KH, self.KW = N, H, W, Ci, Co, KH, KW
        self.sh, self.sw = stride
        self.ph, self.pw = pad
        self.dh, self.dw = dil
        self.Ho = (H + 2 * self.ph - self.dh * (KH - 1) - 1) // self.sh + 1
        self.Wo = (W + 2 * self.pw - self.dw * (KW - 1) - 1) // self.sw + 1
        if self.Ho <= 0 or self.Wo <= 0:
            raise ValueError(f"conv output would be empty: {(H, W)} k={(KH, KW)} s={stride} p={pad}")
        self.T = KH * KW
        self.M = N * self.Ho * self.Wo
        self.taps_h = [r * self.dh - self.ph for r in range(KH) for s in range(KW)]
        self.taps_w = [s * self.dw - self.pw for r in range(KH) for s in range(KW)]
        self.is_pointwise = KH == 1 and KW == 1 and stride == (1, 1) and pad == (0, 0)
        self.implicit_fwd = Ci % 64 == 0 and self.T <= 64
        self.implicit_dgrad = Co % 64 == 0 and Ci % 8 == 0 and self.T <= 64
        self.implicit_wgrad = Ci % 64 == 0 and Co % 8 == 0 and self.T <= 64
        self.gather8_fwd = (not self.implicit_fwd) and Ci % 8 == 0 and self.T <= 64
        self.gather8_wgrad = (not self.implicit_wgrad) and Ci % 8 == 0 and Co % 8 == 0 and self.T <= 64
        self.kpad = math.ceil(self.T * Ci / 8) * 8
        self.fwd_geom = dict(n=N, hi=H, wi=W, c=Ci, ho=self.Ho, wo=self.Wo, sh=self.sh, sw=self.sw, tap_c=Ci,
                             dh=self.taps_h, dw=self.taps_w)
        # data-gradient parity classes
        self.classes = []
        for ph in range(self.sh):
            for pw in range(self.sw):
                Hc = -(-(H - ph) // self.sh)
                Wc = -(-(W - pw) // self.sw)
                if Hc <= 0 or Wc <= 0:
                    continue
                dh_, dw_, wt = [], [], []
                for r in range(KH):
                    nh = ph + self.ph - r * self.dh
                    if nh % self.sh:
                        continue
                    for s in range(KW):
                        nw = pw + self.pw - s * self.dw
                        if nw % self.sw:
                            continue
                        dh_.append(nh // self.sh)
                        dw_.append(nw // self.sw)
                        wt.append(r * KW + s)
                self.classes.append(dict(ph=ph, pw=pw, Hc=Hc, Wc=Wc, dh=dh_, dw=dw_, wt=wt))
        nonempty = [c for c in self.classes if c["wt"]]
        # a single class with taps (1x1 / stride-s downsample): its epilogue zero-fills the
        # other s*s-1 positions, so dX needs no separate memset
        # (its s x s cells must cover the whole input: with padding the class with taps can be an
        # odd-offset one whose grid stops one row / column short)
        self.dgrad_zero_siblings = (len(nonempty) == 1 and (self.sh > 1 or self.sw > 1) and self.sh == self.sw
                                    and len(self.classes) == self.sh * self.sw
                                    and nonempty[0]["Hc"] * self.sh >= H and nonempty[0]["Wc"] * self.sw >= W)
        self.dgrad_needs_zero = (not self.dgrad_zero_siblings) and (
            any(len(c["wt"]) == 0 for c in self.classes) or len(self.classes) < self.sh * self.sw)


@lru_cache(maxsize=4096)
def geometry(N, H, W, Ci, Co, KH, KW, stride, pad, dil):
    return ConvGeometry(N, H, W, Ci, Co, KH, KW, stride, pad, dil)


# ------------------------------------------------------------------------------- native
def _im2col(x, g: ConvGeometry, taps_h, taps_w, ho, wo, sh, sw, kpad):
    col = torch.empty((x.shape[0] * ho * wo, kpad), dtype=torch.bfloat16, device=x.device)
    C().im2col(x, col, ho, wo, sh, sw, list(taps_h), list(taps_w), kpad)
    return col


_HALO3 = True  # the 3x3 stride-1 halo kernel (tests switch it off to compare with the implicit GEMM)


def halo3_ok(g: ConvGeometry) -> bool:
    """The 3x3 / stride-1 / pad-1 halo kernel applies (mirror of ``conv3x3_halo_ok`` in
    csrc/kernels/conv3x3.hip: C and Co multiples of 64, a row tiling of <= 256 output pixels
    whose halo fits 384 LDS rows)."""
    if not (_HALO3 and g.KH == 3 and g.KW == 3 and (g.sh, g.sw) == (1, 1) and (g.ph, g.pw) == (1, 1)
            and (g.dh, g.dw) == (1, 1) and g.Ci % 64 == 0 and g.Co % 64 == 0 and g.implicit_fwd):
        return False
    if g.Ci == 64 and g.Co == 64:
        # one 64-channel chunk: the per-tap halo kernel cannot amortise its halo prologue (measured 0.128 vs
        # 0.120 ms for the implicit GEMM at 56x56; a resident-filter variant lost too, profiles/r4/ab_c64_after_atomics.txt)
        return False
    H, W = g.H, g.W
    if H * W <= 256:
        return H * W * max(1, min(256 // (H * W), 384 // ((H + 2) * (W + 2)))) >= 64
    for r in range(min(H, 256 // W), 0, -1):
        if H % r == 0 and (r + 2) * (W + 2) <= 384:
            return r * W >= 64
    return False


_WG3 = True  # 3x3 stride-1 weight gradients on the halo kernel
_WG3_BPC = 2  # workgroups per CU the pixel split aims for
_WG3_SLAB = True  # partial slabs + reduce instead of atomics
_WG3_PP = True  # 512-thread ping-pong form (one workgroup per CU)


@lru_cache(maxsize=None)
def _device_cus(index: int) -> int:
    return torch.cuda.get_device_properties(index).multi_processor_count


@lru_cache(maxsize=1024)
def _wgrad3_plan(N, H, W, Ci, Co, bpc, cus):
    return C().conv3x3_wgrad_plan(N, H, W, Ci, Co, bpc, cus)


def wgrad3_plan(g: ConvGeometry, device=None):
    """(splits, tiles per split) of the 3x3 / stride-1 / pad-1 weight-gradient halo kernel, or None
    (csrc/kernels/conv3x3.hip: C, Co % 64 == 0 and one of its instantiated row tilings)."""
    if not (_WG3 and g.KH == 3 and g.KW == 3 and (g.sh, g.sw) == (1, 1) and (g.ph, g.pw) == (1, 1)
            and (g.dh, g.dw) == (1, 1) and g.Ci % 64 == 0 and g.Co % 64 == 0):
        return None
    idx = torch.cuda.current_device() if device is None else torch.device(device).index or 0
    return _wgrad3_plan(g.N, g.H, g.W, g.Ci, g.Co, 1 if _WG3_PP else _WG3_BPC, _device_cus(idx))


_SPLITK_FWD = True
_SPLITK_MAX_TILES = 512
_SPLITK_WG = 1024  # workgroups the split aims for


def splitk_fwd_ok(g: ConvGeometry) -> bool:
    """Gathered convolutions with few output tiles (<= 512 64x64 tiles: VGG's 2x2 / 4x4 layers,
    ResNet-50 at 7x7 with small batches) and a long K loop: one workgroup per output tile would
    walk taps x channels alone (measured 77 us for VGG-16's 512-channel 2x2 layers on 88
    workgroups), so the K loop is split over workgroups into an fp32 workspace and a finalize pass
    adds bias / ReLU / statistics."""
    if not (_SPLITK_FWD and g.implicit_fwd and g.T * g.Ci >= 1024 and g.Co % 8 == 0) or _det.enabled():
        return False
    return math.ceil(g.M / 64) * math.ceil(g.Co / 64) <= _SPLITK_MAX_TILES


def conv_fwd_native(x, w, g: ConvGeometry, bias=None, relu=False, stats=None, bnr=None):
    """``bnr``: fused BN-backward reduce of the output (a
    stride-1 data-gradient run as a forward conv; see ``gemm.linear_dgrad``) — applied on the halo and
    gathered implicit-GEMM paths, which then set ``bnr["done"]``."""
    y = torch.empty((g.N, g.Ho, g.Wo, g.Co), dtype=torch.bfloat16, device=x.device)
    y2 = y.view(g.M, g.Co)
    if splitk_fwd_ok(g):
        ws = G.splitk_workspace(g.M, g.Co, x.device)
        K = g.T * g.Ci
        tiles = math.ceil(g.M / 64) * math.ceil(g.Co / 64)
        t128 = math.ceil(g.M / 128) * math.ceil(g.Co / 128)
        s128 = min(768 // t128, K // 576)
        if t128 >= 64 and s128 >= 6:
            # enough 128x128 tiles and K depth for >= 6 splits of >= 9 K-tiles in one round at 3 workgroups
            # per CU: partial slabs summed by the finalize (VGG-16's 4x4 512-channel layers: 52 -> 43 us,
            # scripts/r6/vgg_splitk.py)
            r = G.gemm(x, w, ws, g.M, g.Co, K, G.KC_GATHER, G.KC, 0, K, g.Co, G.EPI_F32, geom=g.fwd_geom, tile=0,
                       k_split=math.ceil(K / s128 / 64) * 64, defer_slabs=True, slabs=True)
        else:
            splits = max(2, min(math.ceil(_SPLITK_WG / tiles), K // 512))  # ~4 workgroups per CU, >= 8 K-tiles
            r = G.gemm(x, w, ws, g.M, g.Co, K, G.KC_GATHER, G.KC, 0, K, g.Co, G.EPI_F32, geom=g.fwd_geom, tile=3,
                       k_split=math.ceil(K / splits / 64) * 64, defer_slabs=True)
        if isinstance(r, tuple):  # partial slabs (DDL_SPLITK_SLABS): summed by the finalize itself
            C().splitk_finalize(r[0], y2, g.Co, bias, bool(relu), stats, r[1])
        else:
            C().splitk_finalize(ws, y2, g.Co, bias, bool(relu), stats)
        return y
    fb = (bnr is not None and bias is None and not relu and stats is None and g.Co % 8 == 0
          and bnr["x"].is_contiguous() and not g.is_pointwise and (halo3_ok(g) or g.implicit_fwd))
    if halo3_ok(g):
        G.gemm(x, w, y2, g.M, g.Co, g.T * g.Ci, G.KC_GATHER, G.KC, 0, g.T * g.Ci, g.Co, G.EPI_BF16, bias=bias,
               relu=relu, geom=g.fwd_geom, stats=stats, tile=G.TILE_CONV3, bnr=bnr if fb else None)
    elif g.is_pointwise:
        G.linear_fwd(x.view(g.M, g.Ci), w.view(g.Co, g.Ci), bias=bias, relu=relu, out=y2, stats=stats)
    elif g.implicit_fwd or g.gather8_fwd:
        G.gemm(x, w, y2, g.M, g.Co, g.T * g.Ci, G.KC_GATHER if g.implicit_fwd else G.KC_GATHER8, G.KC, 0,
               g.T * g.Ci, g.Co, G.EPI_BF16, bias=bias, relu=relu, geom=g.fwd_geom, stats=stats,
               bnr=bnr if fb else None)
    else:
        col = _im2col(x, g, g.taps_h, g.taps_w, g.Ho, g.Wo, g.sh, g.sw, g.kpad)
        w2 = w.reshape(g.Co, g.T * g.Ci)
        if g.kpad != g.T * g.Ci:
            w2 = F.pad(w2, (0, g.kpad - g.T * g.Ci))
        G.linear_fwd(col, w2.contiguous(), bias=bias, relu=relu, out=y2, stats=stats)
    if fb:
        bnr["done"] = True
    return y


def _tap_index(cl, device):
    """Device-resident tap-index tensor of a dgrad class (cached: no host->device copy per
    step, which also keeps the backward capturable into a hipGraph)."""
    cache = cl.setdefault("_wt_dev", {})
    key = str(device)
    if key not in cache:
        cache[key] = torch.tensor(cl["wt"], dtype=torch.int64, device=device)
    return cache[key]


def _dgrad_as_forward(g: ConvGeometry):
    """Stride-1 convolutions: dx is a forward convolution of dy with the flipped, transposed
    filter (padding d*(k-1) - p), which runs on the forward implicit-GEMM path (K-contiguous
    weights, no transposed LDS reads) — measured 1.3-1.7x faster than the RC_TAPS data-gradient
    on the ResNet-50 3x3 layers.  Returns the forward geometry, or None when not applicable."""
    if g.sh != 1 or g.sw != 1 or g.is_pointwise:
        return None
    ph, pw = g.dh * (g.KH - 1) - g.ph, g.dw * (g.KW - 1) - g.pw
    if ph < 0 or pw < 0 or g.Co % 8 or g.Ci % 8 or g.T > 64:
        return None
    g2 = geometry(g.N, g.Ho, g.Wo, g.Co, g.Ci, g.KH, g.KW, (1, 1), (ph, pw), (g.dh, g.dw))
    # narrow channel counts (Co % 64 != 0: MNIST's 32-filter convs) run the per-vector-gathered forward
    # (KC_GATHER8) — two launches (filter flip + conv) where the im2col form took four
    if (g2.Ho, g2.Wo) != (g.H, g.W) or not (g2.implicit_fwd or g2.gather8_fwd):
        return None
    return g2


_KC_DGRAD = True  # strided data-gradients read a K-contiguous per-class filter copy (not RC_TAPS)
_WIDE_WGRAD = True
_WGRAD_ROUNDS = 4.0  # gathered weight gradients: split-K workgroup rounds


def _wgrad_tile(M, N, bn_cap):
    return None


def flip_filter(w):
    """[Co, KH, KW, Ci] -> [Ci, KH, KW, Co] with the taps reversed (the transposed conv's filter):
    one HIP pass on the GPU (``filter_taps_transpose``), flip + permute on the CPU."""
    Co, KH, KW, Ci = w.shape
    if use_native(w) and w.dtype == torch.bfloat16:  # batched with the step's other derived filters (ops/derived.py)
        return derived.taps_transpose(w.contiguous(), range(KH * KW - 1, -1, -1), (Ci, KH, KW, Co))
    return w.flip(1, 2).permute(3, 1, 2, 0).contiguous()


def class_filter(w, g: ConvGeometry, cl):
    """K-contiguous filter of one strided data-gradient class: [Ci][taps of the class][Co]."""
    if use_native(w) and w.dtype == torch.bfloat16:
        return derived.taps_transpose(w.contiguous(), cl["wt"], (g.Ci, len(cl["wt"]), g.Co))
    return w.reshape(g.Co, g.T, g.Ci).index_select(1, _tap_index(cl, w.device)).permute(2, 1, 0).contiguous()


_CLASS_BATCH = True  # strided data-gradients: every parity class in one launch (GemmParams::zcls)


def _class_batch(g: ConvGeometry):
    """The z order of the parity classes of a strided data-gradient run as ONE launch (heaviest class
    first, so its workgroups are dispatched first), or None: every class must have taps and the same
    (Hc, Wc) grid (even H, W at stride 2: ResNet-50's three 3x3 / stride-2 layers), at most 4 classes."""
    cached = getattr(g, "_zcls", False)
    if cached is not False:
        return cached
    cls = g.classes
    ok = (_KC_DGRAD and g.implicit_dgrad and (g.sh > 1 or g.sw > 1) and 1 < len(cls) == g.sh * g.sw <= 4
          and all(c["wt"] for c in cls) and len({(c["Hc"], c["Wc"]) for c in cls}) == 1
          and cls[0]["Hc"] * g.sh == g.H and cls[0]["Wc"] * g.sw == g.W)
    order = sorted(cls, key=lambda c: -len(c["wt"])) if ok else None
    g._zcls = order
    return order


def _dgrad_classes_one_launch(dy, w, g: ConvGeometry, order, dx):
    """All parity classes of a strided data-gradient in one launch: blockIdx.z = class, the class's taps
    of one [Ci][taps of all classes][Co] filter copy, its rows scattered to its (oh, ow) cell of dx."""
    taps, dh, dw, tap0, nt, coff = [], [], [], [], [], []
    for c in order:
        tap0.append(len(taps))
        nt.append(len(c["wt"]))
        taps += c["wt"]
        dh += c["dh"]
        dw += c["dw"]
        coff.append((c["ph"] * g.W + c["pw"]) * g.Ci)
    wkc = derived.taps_transpose(w.contiguous(), taps, (g.Ci, len(taps), g.Co))
    Hc, Wc = order[0]["Hc"], order[0]["Wc"]
    Mc = g.N * Hc * Wc
    K = max(nt) * g.Co
    geom = dict(n=g.N, hi=g.Ho, wi=g.Wo, c=g.Co, ho=Hc, wo=Wc, sh=1, sw=1, tap_c=g.Co, dh=dh, dw=dw)
    om = dict(gh=Hc, gw=Wc, hy=g.H, wy=g.W, so=g.sh, oh=0, ow=0, zero=0)
    tile = G.choose_tile(Mc * len(order), g.Ci)
    C().gemm(dy, wkc, dx, Mc, g.Ci, K, G.KC_GATHER, G.KC, 0, len(taps) * g.Co, g.Ci, G.EPI_BF16, tile, K,
             geom=geom, outmap=om, zcount=len(order), cls_tap0=tap0, cls_nt=nt, cls_coff=coff)


def conv_dgrad_native(dy, w, g: ConvGeometry, resid=None, resid_mask=None, bnr=None, rsub=None):
    """dx = conv^T(dy, w) (+ resid, fused into the epilogue when the layout allows; with
    ``resid_mask`` (1x1 / stride 1 only) only where the residual's ReLU bit is set).  ``bnr``:
    fused BN-backward reduction of dx (pointwise convs on the streaming kernel; see
    ``gemm.linear_dgrad``).  ``rsub = (H, W)``: ``resid`` is on the stride-2 subgrid of dx (pointwise
    convs only)."""
    dev = dy.device
    if (resid_mask is not None or rsub is not None) and not g.is_pointwise:
        raise ValueError("resid_mask / rsub are supported for pointwise (1x1, stride 1) data-gradients only")
    if resid is None:
        g2 = _dgrad_as_forward(g)
        if g2 is not None:
            return conv_fwd_native(dy.contiguous(), flip_filter(w), g2, bnr=bnr)
    if g.is_pointwise:
        dx = torch.empty((g.N, g.H, g.W, g.Ci), dtype=torch.bfloat16, device=dev)
        G.linear_dgrad(dy.view(g.M, g.Co), w.view(g.Co, g.Ci), out=dx.view(-1, g.Ci),
                       resid=None if resid is None else resid.view(-1, g.Ci), resid_mask=resid_mask, bnr=bnr,
                       rsub=rsub)
        return dx
    dx = (torch.zeros if g.dgrad_needs_zero else torch.empty)((g.N, g.H, g.W, g.Ci), dtype=torch.bfloat16, device=dev)
    strided = g.sh > 1 or g.sw > 1
    order = _class_batch(g) if (_CLASS_BATCH and dy.is_contiguous() and w.dtype == torch.bfloat16) else None
    for cl in (() if order else g.classes):
        nt = len(cl["wt"])
        if nt == 0:
            continue
        Mc = g.N * cl["Hc"] * cl["Wc"]
        om = None
        if strided:
            om = dict(gh=cl["Hc"], gw=cl["Wc"], hy=g.H, wy=g.W, so=g.sh, oh=cl["ph"], ow=cl["pw"],
                      zero=int(g.dgrad_zero_siblings))
        r = None if (resid is None or strided) else resid.view(-1, g.Ci)
        if g.implicit_dgrad and _KC_DGRAD:
            # the class's taps of the filter, transposed once to K-contiguous [Ci][taps][Co]: the GEMM
            # then reads B with ds_read_b128 like a forward conv (faster than the RC_TAPS layout)
            wkc = class_filter(w, g, cl)
            geom = dict(n=g.N, hi=g.Ho, wi=g.Wo, c=g.Co, ho=cl["Hc"], wo=cl["Wc"], sh=1, sw=1, tap_c=g.Co,
                        dh=cl["dh"], dw=cl["dw"])
            G.gemm(dy, wkc, dx, Mc, g.Ci, nt * g.Co, G.KC_GATHER, G.KC, 0, nt * g.Co, g.Ci, G.EPI_BF16,
                   geom=geom, outmap=om, resid=r, ldr=g.Ci if r is not None else 0)
        elif g.implicit_dgrad:
            geom = dict(n=g.N, hi=g.Ho, wi=g.Wo, c=g.Co, ho=cl["Hc"], wo=cl["Wc"], sh=1, sw=1, tap_c=g.Co,
                        dh=cl["dh"], dw=cl["dw"], wt=cl["wt"])
            G.gemm(dy, w, dx, Mc, g.Ci, nt * g.Co, G.KC_GATHER, G.RC_TAPS, 0, g.T * g.Ci, g.Ci, G.EPI_BF16,
                   geom=geom, outmap=om, b_kdiv=g.Co, b_tap_stride=g.Ci, resid=r, ldr=g.Ci if r is not None else 0)
        else:
            kp = math.ceil(nt * g.Co / 8) * 8
            col = _im2col(dy, g, cl["dh"], cl["dw"], cl["Hc"], cl["Wc"], 1, 1, kp)
            # wperm[ci][t][co] = w[co][wt[t]][ci]
            wsel = w.reshape(g.Co, g.T, g.Ci).index_select(1, _tap_index(cl, dev))
            wperm = wsel.permute(2, 1, 0).reshape(g.Ci, nt * g.Co)
            if kp != nt * g.Co:
                wperm = F.pad(wperm, (0, kp - nt * g.Co))
            wperm = wperm.contiguous()
            G.gemm(col, wperm, dx, Mc, g.Ci, kp, G.KC, G.KC, kp, kp, g.Ci, G.EPI_BF16, outmap=om, resid=r,
                   ldr=g.Ci if r is not None else 0)
    if order:
        _dgrad_classes_one_launch(dy, w, g, order, dx)
    if resid is not None and strided:
        C().add_bf16(dx, resid, dx)
    return dx


def _slab_wgrad_splits(g: ConvGeometry) -> int:
    """Split count of a gathered weight gradient on 128x128 partial slabs (0: not that path): one round of the
    RC x RC_GATHER kernel's 3 resident workgroups per CU, >= 18 K-tiles per split, <= 32 slabs; only for
    >= 24 output tiles whose 128-column blocks stay inside one tap (Ci % 128 == 0)."""
    if g.Ci % 128 or _det.enabled():
        return 0
    t128 = math.ceil(g.Co / 128) * math.ceil(g.T * g.Ci / 128)
    if t128 < 24:
        return 0
    return min((3 * G._CU) // t128, g.M // 1152, 32)


def conv_wgrad_native(dy, x, g: ConvGeometry, gw):
    """gw[Co, KH, KW, Ci] (fp32) += dW."""
    gw2 = gw.view(g.Co, g.T * g.Ci)
    plan = None if g.is_pointwise else wgrad3_plan(g, dy.device)
    if g.is_pointwise:
        G.linear_wgrad(dy.view(g.M, g.Co), x.view(g.M, g.Ci), gw2)
    elif plan is not None:
        # 3x3 / stride 1: halo kernel (csrc/kernels/conv3x3.hip), 64 co x 64 ci x 9 taps per workgroup
        splits, tpb = plan
        slab = _WG3_SLAB or _det.enabled()  # deterministic mode: never the atomic accumulation
        ws = torch.empty(splits * g.Co * 9 * g.Ci, dtype=torch.float32, device=dy.device) if slab else None
        C().conv3x3_wgrad(dy.contiguous(), x.contiguous(), gw, ws, splits, tpb, _WG3_PP)
    elif g.implicit_wgrad and g.Ci < 128 and _WIDE_WGRAD:
        # narrow inputs (64 channels): a 128-wide tile spans two taps, so the tap is resolved per
        # 16-B vector (GATHER8) instead of per tile — twice the MFMA work per LDS fragment read
        G.gemm(dy, x, gw2, g.Co, g.T * g.Ci, g.M, G.RC, G.RC_GATHER8, g.Co, 0, g.T * g.Ci, G.EPI_F32, beta=1.0,
               geom=g.fwd_geom, bn_cap=128, split_rounds=_WGRAD_ROUNDS, tile=_wgrad_tile(g.Co, g.T * g.Ci, 128))
    elif g.implicit_wgrad and _slab_wgrad_splits(g) >= 2:
        # enough 128x128 output tiles (>= 24) for one round of 3 workgroups per CU with >= 2 splits: 128x128
        # tiles on partial slabs, split count filling that round (ResNet-50's strided layers at 28^2 / 14^2:
        # 3x3 115 -> 92 and 107 -> 83 us, 1x1 downsample 92 -> 77 and 92 -> 74 us; scripts/r6/gather_wgrad.py)
        K = g.T * g.Ci
        G.gemm(dy, x, gw2, g.Co, K, g.M, G.RC, G.RC_GATHER, g.Co, 0, K, G.EPI_F32, beta=1.0, geom=g.fwd_geom,
               tile=0, k_split=math.ceil(g.M / _slab_wgrad_splits(g) / 64) * 64, slabs=True)
    elif g.implicit_wgrad:
        # gathered weight gradients are latency-bound per workgroup: 4 rounds of split-K workgroups
        # (measured: 3-16 % faster than 2 on the ResNet-50 3x3 / strided layers)
        G.gemm(dy, x, gw2, g.Co, g.T * g.Ci, g.M, G.RC, G.RC_GATHER, g.Co, 0, g.T * g.Ci, G.EPI_F32, beta=1.0,
               geom=g.fwd_geom, bn_cap=min(128, g.Ci), split_rounds=_WGRAD_ROUNDS,
               tile=_wgrad_tile(g.Co, g.T * g.Ci, min(128, g.Ci)))
    elif g.gather8_wgrad:
        G.gemm(dy, x, gw2, g.Co, g.T * g.Ci, g.M, G.RC, G.RC_GATHER8, g.Co, 0, g.T * g.Ci, G.EPI_F32, beta=1.0,
               geom=g.fwd_geom)
    else:
        col = _im2col(x, g, g.taps_h, g.taps_w, g.Ho, g.Wo, g.sh, g.sw, g.kpad)
        if g.kpad == g.T * g.Ci:
            G.linear_wgrad(dy.view(g.M, g.Co), col, gw2)
        else:
            tmp = torch.zeros((g.Co, g.kpad), dtype=torch.float32, device=dy.device)
            G.linear_wgrad(dy.view(g.M, g.Co), col, tmp)
            gw2.add_(tmp[:, : g.T * g.Ci])


# ------------------------------------------------------------------------------- reference
def conv_ref(x, w, bias, stride, pad, dil, relu=False):
    y = F.conv2d(x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), bias, stride, pad, dil).permute(0, 2, 3, 1)
    if relu:
        y = torch.relu(y)
    return y.contiguous()


# ------------------------------------------------------------------------------- autograd
class _Conv2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, gw, gb, cfg):
        stride, pad, dil, relu, stats, hook, pads = cfg
        N, H, W, Ci = x.shape
        Co, KH, KW, _ = w.shape
        ctx.cfg = cfg
        ctx.native = use_native(x)
        ctx.ci = Ci
        ctx.co = Co
        if ctx.native:
            # 16-B vector granularity: channel counts padded to multiples of 8 with zeros (stem: 3 -> 8,
            # MNIST: 1 -> 8) — the weights in the arena (params.py, ``pads``) or per call, the input by its
            # producer (ops/zpad.py) or one pad pass here
            Cip, Cop = ZP.r8(Ci), ZP.r8(Co)
            if pads is not None:
                w, b, gw, gb = pads
            elif Cip != Ci or Cop != Co:
                w = F.pad(w.detach(), (0, Cip - Ci, 0, 0, 0, 0, 0, Cop - Co))
                b = None if b is None else F.pad(b.detach(), (0, Cop - Co))
                ctx.grad_tmp = True
            x = ZP.padded(x, Cip) if Cip != Ci else x.contiguous()
            g = geometry(N, H, W, Cip, Cop, KH, KW, stride, pad, dil)
            st = stats
            if stats is not None and Cop != Co:  # statistics of the padded filters land in a wider workspace
                st = torch.zeros((stats.shape[0], 2, Cop), dtype=torch.float32, device=x.device)
            y = conv_fwd_native(x, w, g, bias=b, relu=relu, stats=st)
            if st is not stats:
                stats.copy_(st[:, :, :Co])
            ctx.g = g
        else:
            y = conv_ref(x, w.to(x.dtype), None if b is None else b.to(x.dtype), stride, pad, dil, relu)
        ctx.gw, ctx.gb = gw, gb
        ctx.save_for_backward(x, w, b, y if relu else None)
        ctx.needs_dx = ctx.needs_input_grad[0]
        return ZP.logical(y, Co) if ctx.native else y

    @staticmethod
    def backward(ctx, dy):
        x, w, b, y = ctx.saved_tensors
        gw, gb = ctx.gw, ctx.gb
        stride, pad, dil, relu, _, hook, _ = ctx.cfg
        dx = None
        if ctx.native:
            g = ctx.g
            dy = ZP.padded(dy, g.Co) if g.Co != ctx.co else dy.contiguous()
            if getattr(ctx, "grad_tmp", False):  # logical-shape gradient buffers: padded temporaries
                tgw = None if gw is None else torch.zeros((g.Co, g.KH, g.KW, g.Ci), dtype=torch.float32, device=dy.device)
                tgb = None if gb is None else torch.zeros(g.Co, dtype=torch.float32, device=dy.device)
            else:
                tgw, tgb = gw, gb
            with on_grad_stream(dy.device, dy, x, default=False):  # parameter gradients beside the data-gradient
                if relu:
                    d2 = torch.empty_like(dy)
                    if tgb is not None:  # ReLU backward fused into the bias-gradient sweep
                        C().bias_grad(dy, tgb, g.Co, True, y, d2)
                    else:
                        C().relu_bwd(dy, y, d2)
                    dy = d2
                elif tgb is not None:
                    C().bias_grad(dy, tgb, g.Co, True)
                if tgw is not None:
                    conv_wgrad_native(dy, x, g, tgw)
            if tgw is not gw and gw is not None:
                gw.add_(tgw[: ctx.co, ..., : ctx.ci])
            if tgb is not gb and gb is not None:
                gb.add_(tgb[: ctx.co])
            if ctx.needs_dx:
                dx = ZP.logical(conv_dgrad_native(dy, w, g), ctx.ci)
        else:
            dy = dy.contiguous()
            fn = lambda xx, ww, bb: conv_ref(xx, ww, bb, stride, pad, dil, relu)
            bb = None if b is None else b.to(x.dtype)
            gx, gww, gbb = ref_grads(fn, [x, w.to(x.dtype), bb], dy)
            accumulate(gw, gww)
            accumulate(gb, gbb)
            dx = gx if ctx.needs_dx else None
        if hook is not None:
            hook()
        return dx, None, None, None, None, None


def conv2d(x, w, bias=None, *, stride=1, padding=0, dilation=1, relu=False, grad_w=None, grad_b=None, stats=None,
           on_grad=None, padded=None):
    """NHWC conv.  ``w``: [Co, KH, KW, Ci] compute-dtype weights; ``grad_w``/``grad_b``:
    fp32 buffers that receive ``+= dW``/``+= db`` in backward; ``stats``: optional
    [32, 2, Co] fp32 workspace receiving fused per-channel sum / sum-of-squares
    (GPU); ``on_grad``: callback fired once the parameter gradients are final; ``padded``:
    (weight, bias, weight grad, bias grad) zero-padded arena storage (channels rounded up to multiples
    of 8, ``models/params.py``) that the GPU path uses in place of the logical tensors."""
    cfg = (_pair(stride), _pair(padding), _pair(dilation), bool(relu), stats, on_grad, padded)
    return _Conv2dFn.apply(x, w, bias, grad_w, grad_b, cfg)
