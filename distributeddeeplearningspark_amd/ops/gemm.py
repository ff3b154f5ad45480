"""Python front of the MFMA implicit-GEMM kernel family (``csrc/include/ddl_gemm_kernel.h``).

Semantics: ``C[m][n] = alpha * sum_k A(m,k) * B(n,k)`` with each operand either
K-contiguous (``KC``: ``ptr + r*ld + k``) or row-contiguous (``RC``: ``ptr + k*ld + r``).
So  ``Y = X @ W.T`` (Linear fwd)   = KC x KC,
    ``dX = dY @ W``   (Linear dgrad) = KC x RC,
    ``dW = dY.T @ X`` (Linear wgrad) = RC x RC,
without materialising any transpose: the kernel reads RC operands with
``ds_read_b64_tr_b16`` (hardware LDS transpose).
"""
from __future__ import annotations

import math

import torch

from . import determinism as _det
from ._native import C

KC, RC, KC_GATHER, RC_GATHER, RC_TAPS, KC_GATHER8, RC_GATHER8 = 0, 1, 2, 3, 4, 5, 6
EPI_BF16, EPI_F32, EPI_F32_ATOMIC = 0, 1, 2
TILE256 = 4  # 256x256 ping-pong kernel (csrc/include/ddl_gemm256.h): plain KC/RC operands, K % 64 == 0
TILE_STREAM = 5  # weight-stationary streaming kernel (csrc/kernels/gemm_stream.hip): K in {64, 128, 256}
TILE_CONV3 = 6  # 3x3 stride-1 halo convolution (csrc/kernels/conv3x3.hip): KC_GATHER x KC, no split-K
_TILES = {0: (128, 128), 1: (128, 64), 2: (64, 128), 3: (64, 64), TILE256: (256, 256), TILE_STREAM: (64, 256),
          TILE_CONV3: (224, 128)}
_ONE_PER_CU = (TILE256,)  # kernels running one workgroup per CU
_CU = 256
import os as _os

# Measured (scripts/bench_gemm.py, random bf16): the 256x256 kernel wins on large-K, large-M/N
# GEMMs (8192^3: ~1045 vs ~810 TF for the 128-tile kernel) but loses on the BERT / ResNet
# shapes (K <= 3072 with <= 2.25 workgroup rounds), so it is opt-in (DDL_GEMM256=1) and
# auto-selected only for GEMMs with many tiles AND a long K loop.
_USE256 = "auto"


_USE_STREAM = "1"
# 128x128 tiles per CU below which choose_tile shrinks the tile (one CU holds up to 4 blocks)
_TILE_FILL = 2.0
# Linear data-gradients with at least this many rows use a transposed weight copy (KC x KC GEMM)
_WT_MIN_M = 4096
_LINEAR_WGRAD_ROUNDS = 1.0
# split-K fp32 GEMMs (weight gradients): workgroup rounds to aim for; every split adds one fp32
# atomic per output element, so more rounds trade atomics for parallelism
_SPLIT_ROUNDS = 2.0


def stream_panel(N: int, K: int) -> int:
    """Panel width of the streaming kernel for (N, K) (mirror of ``gemm_stream_panel``), 0 if n/a."""
    if K not in (64, 128, 256):
        return 0
    max_nb = 128 if K == 256 else 256
    nb = max_nb
    while nb >= 64:
        if N % nb == 0 and (N == nb or nb == max_nb):
            return nb
        nb //= 2
    return 0


def use_stream(M, N, K, a_mode, b_mode, epi, lda, ldc, *, outmap=None, aux=None, drop_p=0.0, relu=0, beta=0.0,
               resid=None, ldr=0) -> bool:
    """Skinny-K streaming kernel: ResNet 1x1 convolutions and their data-gradients at large M
    (memory-bound; the 128-tile kernel writes 32-B segments and re-stages the weights per tile)."""
    if _USE_STREAM == "0" or a_mode != KC or b_mode not in (KC, RC) or epi != EPI_BF16:
        return False
    if outmap is not None or aux is not None or drop_p or int(relu) > ACT_RELU or beta:
        return False
    if M < 16384 or not stream_panel(N, K) or lda % 8 or ldc % 8 or (resid is not None and ldr % 4):
        return False
    return True


def use_tile256(M: int, N: int, K: int, a_mode: int, b_mode: int, epi: int) -> bool:
    """The 256x256 kernel pays off when its tiles (times split-K for fp32 outputs) fill the chip."""
    if _USE256 == "0" or a_mode > RC or b_mode > RC or K % 64 or M < 128 or N < 128:
        return False
    tiles = math.ceil(M / 256) * math.ceil(N / 256)
    if _USE256 == "1":
        return tiles >= _CU // 2
    return epi == EPI_BF16 and tiles >= 4 * _CU and K >= 4096


def choose_tile(M: int, N: int, bn_cap: int = 128) -> int:
    bn = 128 if (N > 64 and bn_cap >= 128) else 64
    bm = 128 if M > 64 else 64
    if bm == 128 and bn == 128 and math.ceil(M / 128) * math.ceil(N / 128) < _TILE_FILL * _CU:
        # not enough tiles to fill 256 CUs twice: shrink the tile along the larger extent
        bm = 64 if M <= N else 128
        bn = 64 if M > N else 128
    for tid, (tm, tn) in _TILES.items():
        if (tm, tn) == (bm, bn):
            return tid
    return 3


def choose_split(M: int, N: int, K: int, tile: int, allow: bool, rounds: float | None = None) -> int:
    """Return k_split (elements, multiple of 64).  ``rounds``: workgroup rounds to aim for."""
    kfull = max(64, math.ceil(K / 64) * 64)
    if not allow:
        return kfull
    bm, bn = _TILES[tile]
    tiles = math.ceil(M / bm) * math.ceil(N / bn)
    per_cu = 1 if tile in _ONE_PER_CU else 2  # resident workgroups per CU
    if tiles >= per_cu * _CU or K < 1024:
        return kfull
    splits = min(math.ceil((rounds or _SPLIT_ROUNDS) * per_cu * _CU / tiles), max(1, K // 512))
    ks = math.ceil(K / splits / 64) * 64
    return max(64, ks)


def gemm(a, b, c, M, N, K, a_mode, b_mode, lda, ldb, ldc, epi, *, alpha=1.0, beta=0.0, bias=None, resid=None,
         ldr=0, relu=False, geom=None, outmap=None, b_kdiv=0, b_tap_stride=0, stats=None, tile=None, k_split=None,
         bn_cap=128, aux=None, drop_p=0.0, drop_seed=0, split_rounds=None, resid_mask=None, bnr=None, rsub=None,
         slabs=None, defer_slabs=False):
    """Raw launcher with automatic tile / split-K choice.  ``slabs``: force (True) or forbid (False) the
    partial-slab split-K path of fp32 outputs (default: deterministic mode or DDL_SPLITK_SLABS);
    ``defer_slabs``: when that path is taken, skip the reduce and return ``(slabs, splits)`` for a
    consumer that sums them itself (``splitk_finalize``).

    With ``epi == EPI_F32`` and a split-K decomposition the launch switches to the
    atomic epilogue, which *accumulates* into ``c``: callers that need ``c = A@B``
    must pass a zeroed ``c`` (the gradient arena is zeroed once per step) or
    ``beta == 1`` semantics.
    """
    if tile is None:
        if use_stream(M, N, K, a_mode, b_mode, epi, lda, ldc, outmap=outmap, aux=aux, drop_p=drop_p, relu=relu,
                      beta=beta, resid=resid, ldr=ldr):
            tile = TILE_STREAM
        elif outmap is None and bnr is None and use_tile256(M, N, K, a_mode, b_mode, epi):
            tile = TILE256
        elif epi == EPI_F32 and a_mode <= RC and b_mode <= RC and big_wgrad(M, N, K) and _SPLITK_SLABS_MODE != "0":
            tile = 0  # 128x128 + split-K slabs (see _SPLITK_SLABS_MODE)
        else:
            tile = choose_tile(M, N, bn_cap)
    if (k_split is None and tile == 0 and epi == EPI_F32 and a_mode == RC and b_mode == RC and big_wgrad(M, N, K)
            and _SPLITK_SLABS_MODE == "auto" and slabs is not False):
        k_split = slab_split(M, N, K)
    if k_split is None:
        k_split = choose_split(M, N, K, tile, allow=(epi != EPI_BF16), rounds=split_rounds)
    split_stride = 0
    if k_split < K and epi != EPI_F32 and _det.enabled():
        k_split = max(64, math.ceil(K / 64) * 64)  # deterministic mode: no atomic split-K partial sums
    out, slab_beta = c, None
    if epi == EPI_F32 and k_split < K:
        if beta not in (0.0, 1.0):
            raise ValueError("split-K fp32 gemm supports beta in {0,1} (beta=0 needs a zeroed C)")
        auto = _SPLITK_SLABS_MODE == "auto" and tile == 0 and big_wgrad(M, N, K) and math.ceil(K / k_split) <= 32
        use_slabs = (_det.enabled() or _SPLITK_SLABS or auto) if slabs is None else (slabs or _det.enabled())
        if tile in (0, 1, 2, 3) + _ONE_PER_CU and use_slabs:
            # partial slabs (plain stores) + an ordered reduce: deterministic, and the slab stores run at
            # the HBM store rate where fp32 atomics run at ~1.3 TB/s (GemmParams::split_stride)
            splits = math.ceil(K / k_split)
            out, split_stride, slab_beta, ldc_c = _slab_workspace(splits * M * N, c.device), M * N, beta, ldc
            ldc, beta = N, 0.0
        else:
            epi = EPI_F32_ATOMIC
    if bnr is not None:  # fused BN-backward reduce of the output (see linear_dgrad / GemmParams.bnr_*)
        if tile in _ONE_PER_CU:
            raise ValueError("bnr: not on the 256-row kernels")
        stats = bnr["ws"]
    C().gemm(a, b, out, M, N, K, a_mode, b_mode, lda, ldb, ldc, epi, tile, k_split, alpha, beta, bias, resid, ldr,
             int(relu), geom, outmap, b_kdiv, b_tap_stride, stats, aux, float(drop_p), int(drop_seed), resid_mask,
             None if bnr is None else bnr["x"], None if bnr is None else bnr.get("mask"),
             None if bnr is None else bnr["mean"], *(rsub or (0, 0)), None if bnr is None else bnr.get("scale"),
             None if bnr is None else bnr.get("shift"), split_stride)
    if split_stride:
        if defer_slabs:
            return out, math.ceil(K / k_split)
        C().slab_reduce(out, math.ceil(K / k_split), c, M, N, ldc_c, float(slab_beta))
    return c


# DDL_SPLITK_SLABS=1: fp32 split-K GEMMs (weight gradients) through partial slabs instead of fp32 atomics;
# "auto" (default): slabs for the large-output long-reduction weight gradients (big_wgrad), atomics for the
# rest — measured (profiles/r4/gemm_sweep.txt): BERT-base weight gradients on 128x128 tiles 536-649 TF/s
# with atomics, 638-724 with slabs; ResNet-50 1x1 weight gradients (hundreds of splits of a small output,
# where the slab reduce has too little parallelism) 283 / 570 with atomics, 166 / 532 with slabs
_SPLITK_SLABS_MODE = _os.environ.get("DDL_SPLITK_SLABS", "auto")
_SPLITK_SLABS = _SPLITK_SLABS_MODE == "1"


def big_wgrad(M: int, N: int, K: int) -> bool:
    """An fp32 GEMM with at least 2^19 outputs over a long reduction (BERT's QKV / FFN / attention-output weight
    gradients): 128x128 tiles split over K into partial slabs beat smaller tiles with fp32 atomics."""
    return M * N >= (1 << 19) and K >= 8192 and M >= 512 and N >= 512


def slab_split(M: int, N: int, K: int) -> int:
    """k_split of a 128x128 RC x RC partial-slab GEMM (weight gradient): as many splits as fill ONE round of
    the kernel's 3 resident workgroups per CU, each split at least 18 K-tiles (1,152) deep.  BERT-base at
    16,384 tokens (`scripts/r6/wgrad_splits.py`, TF/s incl. the slab reduce): QKV 7 splits 716 (was 10: 644),
    FFN 5 splits 772 / 789 (was 8: 736 / 740), attention output 14 splits 513 (was 64x128 + atomics: 443)."""
    tiles = math.ceil(M / 128) * math.ceil(N / 128)
    splits = max(1, min((3 * _CU) // tiles, K // 1152))
    return max(64, math.ceil(K / splits / 64) * 64)
_SLAB_WS: dict = {}


def _slab_workspace(n, device):
    """Per-(device, stream, replica scope) fp32 workspace of split-K partial slabs (grown on demand; calls on
    one stream are ordered, so one buffer per stream is enough)."""
    from . import scope as _scope

    key = (str(device), torch.cuda.current_stream(device).cuda_stream if device.type == "cuda" else 0, _scope.tag())
    ws = _SLAB_WS.get(key)
    if ws is None or ws.numel() < n:
        ws = _SLAB_WS[key] = torch.empty(max(n, 1 << 20), dtype=torch.float32, device=device)
    return ws[:n]


# ----------------------------------------------------------------------------------------
# 2-D helpers (row-major tensors)
# ----------------------------------------------------------------------------------------
ACT_NONE, ACT_RELU, ACT_GELU, ACT_GELU_BWD = 0, 1, 2, 3


def linear_fwd(x2, w, bias=None, relu=False, out=None, resid=None, stats=None, act=None, aux=None, drop_p=0.0,
               drop_seed=0):
    """y[M,N] = x2[M,K] @ w[N,K]^T (+bias) -> act -> dropout (+resid) -> bf16.

    ``act``: ACT_RELU / ACT_GELU (``aux`` receives the bf16 pre-activation)."""
    M, K = x2.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=x2.device)
    act = (ACT_RELU if relu else ACT_NONE) if act is None else act
    tiles = math.ceil(M / 64) * math.ceil(N / 64)
    if (K >= 1024 and tiles <= _SKINNY_FWD_TILES and act <= ACT_RELU and resid is None and stats is None and aux is None
            and not drop_p and N % 8 == 0 and out.is_contiguous() and x2.device.type == "cuda" and not _det.enabled()):
        # a few output tiles over a long reduction (a Dense on a flattened feature map at a small batch:
        # MNIST's [16, 4608] x [4608, 232] is 4 tiles of 72 K-steps): the reduction is split over
        # workgroups into an fp32 workspace, and one finalize pass adds the bias / ReLU and rounds
        ws = splitk_workspace(M, N, x2.device)
        splits = max(2, min(math.ceil(256 / tiles), K // 256))
        r = gemm(x2, w, ws, M, N, K, KC, KC, x2.stride(0), w.stride(0), N, EPI_F32, tile=3,
                 k_split=math.ceil(K / splits / 64) * 64, defer_slabs=True)
        if isinstance(r, tuple):
            C().splitk_finalize(r[0], out, N, bias, act == ACT_RELU, None, r[1])
        else:
            C().splitk_finalize(ws, out, N, bias, act == ACT_RELU, None)
        return out
    return gemm(x2, w, out, M, N, K, KC, KC, x2.stride(0), w.stride(0), out.stride(0), EPI_BF16, bias=bias, relu=act,
                resid=resid, ldr=(resid.stride(0) if resid is not None else 0), stats=stats, aux=aux, drop_p=drop_p,
                drop_seed=drop_seed)


_SPLITK_WS = {}
_SKINNY_FWD_TILES = 16  # 64x64 output tiles at or below which a long-K bf16 Linear forward splits K


def splitk_workspace(M, N, device):
    """Persistent zeroed fp32 [M, N] accumulator of a split-K bf16 GEMM: ``splitk_finalize`` zeroes
    it again as it reads it, so consecutive calls (one stream) need no fill launch."""
    from . import scope as _scope

    key = (M, N, str(device) + _scope.tag())
    ws = _SPLITK_WS.get(key)
    if ws is None:
        ws = _SPLITK_WS[key] = torch.zeros((M, N), dtype=torch.float32, device=device)
    return ws


_SPLITK_DGRAD = True


def linear_dgrad(dy, w, out=None, resid=None, gelu_pre=None, stats=None, resid_mask=None, bnr=None, rsub=None):
    """dx[M,K] = dy[M,N] @ w[N,K] (* gelu'(gelu_pre)) (+resid) -> bf16 (w read row-contiguous).

    ``stats`` ([32, 2, K] fp32, zeroed): per-column sums / sums of squares of the output;
    ``resid_mask``: uint8 ReLU bit mask of ``resid`` (bn.hip mode-3 layout) — only the masked
    residual is added; ``bnr`` = {"x", "mask", "mean", "ws"} (mode-3 bit mask) or {"x", "scale",
    "shift", "mean", "ws"} (mode 2: ReLU recomputed from x): the GEMM's epilogue also accumulates the
    BatchNorm-backward partial sums of the output (``GemmParams.bnr_*``) into ``ws`` and
    ``bnr["done"]`` is set — the consumer BN then skips its reduce sweep.  Where no kernel can
    (mode 2 with a residual on the streaming kernel, split-K) ``bnr`` is left untouched.  ``rsub = (H, W)``: the rows are an
    [N][H][W] grid and ``resid`` lives on its stride-2 subgrid (``GemmParams.rsub_h``)."""
    M, N = dy.shape
    K = w.shape[1]
    if out is None:
        out = torch.empty((M, K), dtype=torch.bfloat16, device=dy.device)
    act = ACT_GELU_BWD if gelu_pre is not None else ACT_NONE
    ldr = resid.stride(0) if resid is not None else 0
    tiles = math.ceil(M / 64) * math.ceil(K / 64)
    if (_SPLITK_DGRAD and not _det.enabled() and gelu_pre is None and resid is None and rsub is None and N >= 4096 and tiles <= 1024 and K % 8 == 0
            and out.is_contiguous() and out.dtype == torch.bfloat16 and dy.device.type == "cuda"):
        # few output tiles over a long reduction (BERT's MLM decoder: [masked tokens, 768] over the
        # 30,522-word vocabulary ran on 240 workgroups of ~480 K-steps): split the reduction over
        # workgroups into an fp32 workspace, then round (+ statistics) in one finalize pass
        ws = splitk_workspace(M, K, dy.device)
        t128 = math.ceil(M / 128) * math.ceil(K / 128)
        if 2 * t128 <= 3 * _CU:
            # 128x128 tiles on partial slabs, as many splits as fill one round of the kernel's 3 resident
            # workgroups per CU (the decoder: 120 tiles x 6 splits): 205 -> 141 us vs 64x64 tiles + fp32
            # atomics (scripts/r6/decoder_dgrad.py); the finalize sums the slabs in split order
            splits = max(2, min((3 * _CU) // t128, N // 1152))
            r = gemm(dy, w, ws, M, K, N, KC, RC, dy.stride(0), w.stride(0), K, EPI_F32, tile=0,
                     k_split=math.ceil(N / splits / 64) * 64, defer_slabs=True, slabs=True)
        else:
            splits = max(2, min(math.ceil(2048 / tiles), N // 512))
            r = gemm(dy, w, ws, M, K, N, KC, RC, dy.stride(0), w.stride(0), K, EPI_F32, tile=3,
                     k_split=math.ceil(N / splits / 64) * 64, defer_slabs=True)
        if isinstance(r, tuple):  # partial slabs (DDL_SPLITK_SLABS): summed by the finalize itself
            C().splitk_finalize(r[0], out, K, None, False, stats, r[1])
        else:
            C().splitk_finalize(ws, out, K, None, False, stats)
        return out
    if M >= _WT_MIN_M and not use_stream(M, K, N, KC, RC, EPI_BF16, dy.stride(0), out.stride(0), aux=gelu_pre,
                                         relu=act, resid=resid, ldr=ldr):
        # transpose the (small) weight once so the GEMM reads B K-contiguous with ds_read_b128 instead
        # of paired transposed LDS reads: the BERT-size data-gradients run ~1.4x faster this way
        wt = transpose(w)
        fb = _bnr_plain_ok(bnr, stats, resid, gelu_pre, K)
        gemm(dy, wt, out, M, K, N, KC, KC, dy.stride(0), wt.stride(0), out.stride(0), EPI_BF16, resid=resid,
             ldr=ldr, relu=act, aux=gelu_pre, stats=stats, resid_mask=resid_mask, rsub=rsub, bnr=bnr if fb else None)
        if fb:
            bnr["done"] = True
        return out
    if (bnr is not None and stats is None and ("scale" not in bnr or (resid is None and rsub is None))
            and use_stream(M, K, N, KC, RC, EPI_BF16, dy.stride(0), out.stride(0), aux=gelu_pre, relu=act,
                           resid=resid, ldr=ldr)):
        gemm(dy, w, out, M, K, N, KC, RC, dy.stride(0), w.stride(0), out.stride(0), EPI_BF16, resid=resid, ldr=ldr,
             relu=act, aux=gelu_pre, resid_mask=resid_mask, tile=TILE_STREAM, bnr=bnr, rsub=rsub)
        bnr["done"] = True
        return out
    fb = _bnr_plain_ok(bnr, stats, resid, gelu_pre, K) and not use_stream(
        M, K, N, KC, RC, EPI_BF16, dy.stride(0), out.stride(0), aux=gelu_pre, relu=act, resid=resid, ldr=ldr)
    gemm(dy, w, out, M, K, N, KC, RC, dy.stride(0), w.stride(0), out.stride(0), EPI_BF16, resid=resid,
         ldr=ldr, relu=act, aux=gelu_pre, stats=stats, resid_mask=resid_mask, rsub=rsub, bnr=bnr if fb else None)
    if fb:
        bnr["done"] = True
    return out


def _bnr_plain_ok(bnr, stats, resid, gelu_pre, ncols) -> bool:
    """The LDS-DMA GEMM's EPI_BF16_BNR epilogue can take this data-gradient's BN-backward reduce (a residual
    included: 8-B aligned rows of 4-element multiples, as its 4-column fragment loads read it)."""
    return (bnr is not None and stats is None and gelu_pre is None and ncols % 8 == 0 and bnr["x"].is_contiguous()
            and (resid is None or (resid.stride(0) % 4 == 0 and resid.data_ptr() % 8 == 0)))


def transpose(w):
    """Contiguous bf16 ``w.t()`` from the LDS-tiled HIP transpose (shapes multiple of 8; others
    take torch's copy, which the ATen strided-copy kernel runs ~5x slower at BERT weight sizes)."""
    R, Cc = w.shape
    if w.stride(1) != 1 or R % 8 or Cc % 8 or w.stride(0) % 8:
        return w.t().contiguous()
    if w.is_contiguous():  # batched with the step's other derived weights (ops/derived.py)
        from . import derived

        return derived.taps_transpose(w, (0,), (Cc, R))
    out = torch.empty((Cc, R), dtype=w.dtype, device=w.device)
    C().transpose_bf16(w, out)
    return out


def linear_wgrad(dy, x2, gw):
    """gw[N,K] += dy[M,N]^T @ x2[M,K]  (fp32 accumulation into the gradient arena)."""
    M, N = dy.shape
    K = x2.shape[1]
    # measured on the ResNet-50 1x1 weight gradients: one workgroup round (half the fp32 atomics
    # of two rounds) is 5-15 % faster — these GEMMs are bound by the split-K atomics, not MFMA
    # (the large BERT weight gradients, on 128x128 tiles with partial slabs, take two rounds: 8 splits
    # measured 642-739 TF/s vs 629-689 at one round, profiles/r4/wgrad_slabs_ab.txt)
    rounds = None if (big_wgrad(N, K, M) and _SPLITK_SLABS_MODE == "auto") else _LINEAR_WGRAD_ROUNDS
    return gemm(dy, x2, gw, N, K, M, RC, RC, dy.stride(0), x2.stride(0), gw.stride(0), EPI_F32, beta=1.0,
                split_rounds=rounds)


def matmul(a, b, trans_a=False, trans_b=False, out=None, alpha=1.0):
    """General bf16 matmul op(a) @ op(b) -> bf16 using the KC/RC operand modes."""
    M = a.shape[1] if trans_a else a.shape[0]
    K = a.shape[0] if trans_a else a.shape[1]
    N = b.shape[0] if trans_b else b.shape[1]
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    a_mode = RC if trans_a else KC
    # B(n,k): op(b)[k][n]; trans_b -> b[n][k] is K-contiguous
    b_mode = KC if trans_b else RC
    return gemm(a, b, out, M, N, K, a_mode, b_mode, a.stride(0), b.stride(0), out.stride(0), EPI_BF16, alpha=alpha)
