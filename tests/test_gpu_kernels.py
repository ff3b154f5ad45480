"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op.

Inputs are rounded to bf16 first, then the reference runs in fp32 on those exact
values; tolerances reflect bf16 outputs (rel ~1e-2) and fp32 accumulation.
Operands are asymmetric random data (catches transposed C/D maps).
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _C():
    from distributeddeeplearningspark_amd.ops._native import C

    return C()


def rnd(*shape, scale=1.0, dtype=torch.bfloat16, seed=None):
    g = torch.Generator(device="cpu")
    g.manual_seed(seed if seed is not None else (hash(shape) & 0xFFFF))
    return (torch.randn(*shape, generator=g) * scale).to(dtype).to(DEV)


def close(a, b, rtol=2e-2, atol=2e-2, what=""):
    a = a.float().cpu()
    b = b.float().cpu()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = (err > tol).float().mean().item()
    rel = (err.norm() / (b.norm() + 1e-12)).item()
    assert bad < 1e-3 and rel < 2e-2, f"{what}: frac_bad={bad:.2e} rel_l2={rel:.2e} max_err={err.max().item():.3e}"


# ----------------------------------------------------------------------------- GEMM
@pytest.mark.parametrize("M,N,K", [(256, 256, 256), (200, 72, 136), (1000, 384, 64), (64, 1000, 2048), (8, 16, 8)])
@pytest.mark.parametrize("a_rc", [False, True])
@pytest.mark.parametrize("b_rc", [False, True])
@pytest.mark.parametrize("tile", [0, 1, 2, 3])
def test_gemm_layouts(M, N, K, a_rc, b_rc, tile):
    from distributeddeeplearningspark_amd.ops import gemm as G

    if (a_rc and M % 8) or (b_rc and N % 8):
        pytest.skip("row-contiguous operands need a multiple of 8 rows")
    A = rnd(M, K, seed=1)          # logical A [M,K]
    B = rnd(N, K, seed=2)          # logical B [N,K]
    ref = A.float() @ B.float().T
    a_t = A.T.contiguous() if a_rc else A.contiguous()
    b_t = B.T.contiguous() if b_rc else B.contiguous()
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    G.gemm(a_t, b_t, out, M, N, K, G.RC if a_rc else G.KC, G.RC if b_rc else G.KC, a_t.stride(0), b_t.stride(0), N,
           G.EPI_BF16, tile=tile)
    close(out, ref, what=f"gemm a_rc={a_rc} b_rc={b_rc} tile={tile}")


def test_gemm_identity_asymmetric():
    from distributeddeeplearningspark_amd.ops import gemm as G

    n = 64
    A = torch.eye(n, dtype=torch.bfloat16, device=DEV)
    B = (torch.arange(n * n, device=DEV).reshape(n, n) % 97).to(torch.bfloat16)  # B[n][k], asymmetric
    out = torch.empty(n, n, dtype=torch.bfloat16, device=DEV)
    G.gemm(A, B, out, n, n, n, G.KC, G.KC, n, n, n, G.EPI_BF16)
    assert torch.equal(out.float(), B.float().T), "C/D map transposed"


def test_gemm_epilogues_and_splitk():
    from distributeddeeplearningspark_amd.ops import gemm as G

    M, N, K = 512, 192, 1024
    A, B = rnd(M, K, seed=3), rnd(N, K, seed=4)
    bias = torch.randn(N, device=DEV)
    res = rnd(M, N, seed=5)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    G.gemm(A, B, out, M, N, K, G.KC, G.KC, K, K, N, G.EPI_BF16, bias=bias, resid=res, ldr=N, relu=True)
    ref = torch.relu(A.float() @ B.float().T + bias + res.float())
    close(out, ref, what="bias+resid+relu")
    # fp32 split-K accumulate (wgrad-shaped: small M,N, huge K)
    M2, N2, K2 = 64, 576, 50176
    dy, x = rnd(K2, M2, seed=6), rnd(K2, N2, seed=7)
    gw = torch.full((M2, N2), 0.5, device=DEV)
    G.gemm(dy, x, gw, M2, N2, K2, G.RC, G.RC, M2, N2, N2, G.EPI_F32, beta=1.0)
    ref2 = 0.5 + dy.float().T @ x.float()
    close(gw, ref2, rtol=1e-3, atol=1e-2, what="split-K fp32 accumulate")


def test_gemm_fused_stats():
    from distributeddeeplearningspark_amd.ops import gemm as G

    M, N, K = 3000, 128, 192
    A, B = rnd(M, K, seed=8), rnd(N, K, seed=9)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    st = torch.zeros(32, 2, N, device=DEV)
    G.gemm(A, B, out, M, N, K, G.KC, G.KC, K, K, N, G.EPI_BF16, stats=st)
    s = st.sum(0)
    o = out.float()
    close(s[0], o.sum(0), rtol=1e-3, atol=1e-1, what="fused sum")
    close(s[1], (o * o).sum(0), rtol=1e-3, atol=1e-1, what="fused sumsq")


# ----------------------------------------------------------------------------- conv
CONV_CASES = [
    # N, H, W, Ci, Co, k, stride, pad
    (2, 14, 14, 64, 64, 3, 1, 1),
    (2, 15, 15, 64, 128, 3, 2, 1),
    (2, 14, 14, 128, 64, 3, 2, 1),  # even grid: the four parity classes in one launch (GemmParams::zcls)
    (2, 14, 14, 256, 512, 1, 2, 0),
    (2, 7, 7, 128, 64, 1, 1, 0),
    (2, 32, 32, 3, 64, 7, 2, 3),   # stem: im2col path
    (4, 28, 28, 1, 32, 3, 1, 0),   # MNIST conv1
    (4, 26, 26, 32, 32, 3, 1, 0),  # MNIST conv2 (im2col fwd / implicit-less dgrad)
    (2, 9, 9, 128, 128, 3, 1, 1),
    (4, 4, 4, 256, 128, 3, 1, 1),  # few output tiles: split-K forward (fp32 workspace + finalize)
    (8, 2, 2, 512, 512, 3, 1, 1),  # VGG-16's 2x2 layers
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_bwd(case):
    from distributeddeeplearningspark_amd.ops.conv import conv2d

    N, H, W, Ci, Co, k, s, p = case
    x = rnd(N, H, W, Ci, seed=10)
    w = rnd(Co, k, k, Ci, scale=1.0 / math.sqrt(k * k * Ci), seed=11)
    b = torch.randn(Co, device=DEV) * 0.1
    gw = torch.zeros(Co, k, k, Ci, device=DEV)
    gb = torch.zeros(Co, device=DEV)
    xg = x.clone().requires_grad_(True)
    w_anchor = w.clone().requires_grad_(True)
    y = conv2d(xg, w_anchor, b, stride=s, padding=p, grad_w=gw, grad_b=gb)
    dy = rnd(*y.shape, seed=12)
    y.backward(dy)
    # fp32 reference on the same bf16 values
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.float().permute(0, 3, 1, 2).requires_grad_(True)
    br = b.clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, br, s, p)
    yr.backward(dy.float().permute(0, 3, 1, 2))
    close(y, yr.permute(0, 2, 3, 1), what=f"conv fwd {case}")
    close(xg.grad, xr.grad.permute(0, 2, 3, 1), what=f"conv dgrad {case}")
    close(gw, wr.grad.permute(0, 2, 3, 1), rtol=1e-2, atol=1e-2, what=f"conv wgrad {case}")
    close(gb, br.grad, rtol=1e-2, atol=1e-2, what=f"conv bgrad {case}")


@pytest.mark.parametrize("N,H,Ci,Co", [(2, 14, 128, 64), (4, 28, 64, 128), (3, 8, 256, 512)])
def test_strided_dgrad_classes_one_launch(N, H, Ci, Co, monkeypatch):
    """3x3 / stride-2 data-gradient: the four parity classes as ONE launch (blockIdx.z = class, heaviest
    class first) equal the one-launch-per-class path bit for bit, and the fp32 reference; with and
    without a residual."""
    from distributeddeeplearningspark_amd.ops import conv as CV

    g = CV.geometry(N, H, H, Ci, Co, 3, 3, (2, 2), (1, 1), (1, 1))
    assert CV._class_batch(g) is not None and [len(c["wt"]) for c in CV._class_batch(g)] == [4, 2, 2, 1]
    w = rnd(Co, 3, 3, Ci, scale=1.0 / math.sqrt(9 * Ci), seed=60)
    dy = rnd(N, g.Ho, g.Wo, Co, seed=61)
    r = rnd(N, H, H, Ci, seed=62)
    one = CV.conv_dgrad_native(dy, w, g)
    one_r = CV.conv_dgrad_native(dy, w, g, resid=r)
    monkeypatch.setattr(CV, "_CLASS_BATCH", False)
    per = CV.conv_dgrad_native(dy, w, g)
    assert torch.equal(one, per)
    assert torch.equal(one_r, CV.conv_dgrad_native(dy, w, g, resid=r))
    wr = w.float().permute(0, 3, 1, 2)
    ref = torch.nn.grad.conv2d_input((N, Ci, H, H), wr, dy.float().permute(0, 3, 1, 2), stride=2, padding=1)
    close(one, ref.permute(0, 2, 3, 1), what=f"one-launch strided dgrad {N}x{H}x{Ci}->{Co}")


@pytest.mark.parametrize("M,N,K", [(20000, 256, 64), (600, 512, 128), (4096, 2048, 512)])
def test_dgrad_masked_residual(M, N, K):
    """dx = dy @ w + resid * bit(mask): the identity-shortcut gradient of a ResNet block added
    under the block-output ReLU mask in the data-gradient epilogue (streaming kernel at large M,
    the tile kernels otherwise)."""
    from distributeddeeplearningspark_amd.ops import gemm as G

    dy, w, r = rnd(M, K, seed=40), rnd(K, N, scale=0.1, seed=41), rnd(M, N, seed=42)
    keep = torch.rand(M, N, device=DEV) > 0.5
    # bn.hip mode-3 layout: byte e // 8 holds bit e % 8 of flat element e
    bits = keep.reshape(-1, 8).to(torch.uint8) << torch.arange(8, device=DEV, dtype=torch.uint8)
    mask = bits.sum(1, dtype=torch.uint8)
    out = G.linear_dgrad(dy, w, resid=r, resid_mask=mask)
    ref = dy.float() @ w.float() + r.float() * keep
    close(out, ref, what=f"masked residual dgrad {M}x{N}x{K}")


@pytest.mark.parametrize("slabs", [False, True])
@pytest.mark.parametrize("M", [300, 2458])
def test_linear_dgrad_splitk(M, slabs, monkeypatch):
    """Long-reduction data-gradient on few output tiles (BERT's MLM decoder: masked tokens x 768
    over the vocabulary) runs split-K into the fp32 workspace (or partial slabs summed by the
    finalize): values, statistics, and the workspace left zeroed for the next call (two calls)."""
    from distributeddeeplearningspark_amd.ops import gemm as G

    monkeypatch.setattr(G, "_SPLITK_SLABS", slabs)

    V, H = 8200, 768
    for seed in (50, 52):
        dy, w = rnd(M, V, seed=seed), rnd(V, H, scale=0.02, seed=seed + 1)
        st = torch.zeros(32, 2, H, device=DEV)
        out = G.linear_dgrad(dy, w, stats=st)
        ref = dy.float() @ w.float()
        close(out, ref, what=f"split-K dgrad M={M} seed={seed}")
        o = out.float()
        close(st.sum(0)[0], o.sum(0), rtol=1e-3, atol=1e-2, what="split-K dgrad stats")
    assert G.splitk_workspace(M, H, dy.device).abs().max().item() == 0.0


@pytest.mark.parametrize("N,H,Ci,Co,k", [(64, 14, 512, 512, 3), (64, 14, 1024, 2048, 1), (32, 28, 256, 256, 3)])
def test_gathered_wgrad_on_partial_slabs(N, H, Ci, Co, k):
    """Strided weight gradients with >= 24 128x128 output tiles run on 128x128 partial slabs (one round of
    3 workgroups per CU): against the fp32 reference, accumulating onto an existing gradient."""
    from distributeddeeplearningspark_amd.ops import conv as CV

    p = 1 if k == 3 else 0
    g = CV.geometry(N, H, H, Ci, Co, k, k, (2, 2), (p, p), (1, 1))
    assert CV._slab_wgrad_splits(g) >= 2
    x = rnd(N, H, H, Ci, seed=70)
    dy = rnd(N, g.Ho, g.Wo, Co, seed=71)
    gw0 = torch.randn(Co, k, k, Ci, device=DEV)
    gw = gw0.clone()
    CV.conv_wgrad_native(dy, x, g, gw)
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (Co, Ci, k, k), dy.float().permute(0, 3, 1, 2),
                                      stride=2, padding=p).permute(0, 2, 3, 1)
    close(gw - gw0, ref, rtol=1e-2, atol=1e-2, what=f"slab wgrad {N}x{H}x{Ci}->{Co} k{k}")


@pytest.mark.parametrize("slabs", [False, True])
@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("N,Co", [(16, 256), (256, 512)])
def test_conv_splitk_forward_stats(relu, slabs, N, Co, monkeypatch):
    """Split-K forward of a small-grid conv: bias, ReLU and the fused per-channel statistics of the
    rounded bf16 output ([32, 2, C] sharded sums, as the GEMM epilogue writes them); with partial
    slabs the finalize sums them itself."""
    from distributeddeeplearningspark_amd.ops import conv as CV
    from distributeddeeplearningspark_amd.ops import gemm as G

    monkeypatch.setattr(G, "_SPLITK_SLABS", slabs)

    H, Ci = 4, 512  # N = 256, Co = 512: VGG-16's 4x4 layer, 128x128 tiles on partial slabs (6 splits)
    g = CV.geometry(N, H, H, Ci, Co, 3, 3, (1, 1), (1, 1), (1, 1))
    assert CV.splitk_fwd_ok(g)
    x = rnd(N, H, H, Ci, seed=30)
    w = rnd(Co, 3, 3, Ci, scale=1.0 / math.sqrt(9 * Ci), seed=31)
    b = torch.randn(Co, device=DEV) * 0.1
    st = torch.zeros(32, 2, Co, device=DEV)
    y = CV.conv_fwd_native(x, w, g, bias=b, relu=relu, stats=st)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b, 1, 1).permute(0, 2, 3, 1)
    if relu:
        ref = torch.relu(ref)
    close(y, ref, what="split-K conv fwd")
    o = y.float().reshape(-1, Co)
    close(st.sum(0)[0], o.sum(0), rtol=1e-3, atol=1e-2, what="split-K stats sum")
    close(st.sum(0)[1], (o * o).sum(0), rtol=1e-3, atol=1e-2, what="split-K stats sumsq")


def test_conv_relu_fused():
    from distributeddeeplearningspark_amd.ops.conv import conv2d

    x = rnd(2, 10, 10, 64, seed=13)
    w = rnd(64, 3, 3, 64, scale=0.05, seed=14)
    xg = x.clone().requires_grad_(True)
    y = conv2d(xg, w.clone().requires_grad_(True), None, stride=1, padding=1, relu=True)
    dy = rnd(*y.shape, seed=15)
    y.backward(dy)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = torch.relu(F.conv2d(xr, w.float().permute(0, 3, 1, 2), None, 1, 1))
    yr.backward(dy.float().permute(0, 3, 1, 2))
    close(y, yr.permute(0, 2, 3, 1), what="conv+relu fwd")
    close(xg.grad, xr.grad.permute(0, 2, 3, 1), what="conv+relu dgrad")


# ----------------------------------------------------------------------------- batch norm
@pytest.mark.parametrize("resid,relu", [(False, False), (True, True), (False, True)])
def test_batchnorm(resid, relu):
    from distributeddeeplearningspark_amd.ops.norm import batch_norm

    N, H, W, Cc = 8, 7, 7, 256
    x = (rnd(N, H, W, Cc, seed=16).float() * 2 + 0.5).to(torch.bfloat16)
    r = rnd(N, H, W, Cc, seed=17) if resid else None
    g = torch.rand(Cc, device=DEV) + 0.5
    b = torch.randn(Cc, device=DEV) * 0.1
    rm, rv = torch.zeros(Cc, device=DEV), torch.ones(Cc, device=DEV)
    gg, gbt = torch.zeros(Cc, device=DEV), torch.zeros(Cc, device=DEV)
    xg = x.clone().requires_grad_(True)
    rg = r.clone().requires_grad_(True) if resid else None
    y = batch_norm(xg, g.clone().requires_grad_(True), b, rm, rv, training=True, momentum=0.1, eps=1e-5,
                   resid=rg, relu=relu, grad_gamma=gg, grad_beta=gbt)
    dy = rnd(*y.shape, seed=18)
    y.backward(dy)
    xr = x.float().requires_grad_(True)
    gr, br = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    rr = r.float().requires_grad_(True) if resid else None
    mean = xr.mean((0, 1, 2))
    var = xr.var((0, 1, 2), unbiased=False)
    yr = (xr - mean) / torch.sqrt(var + 1e-5) * gr + br
    if resid:
        yr = yr + rr
    if relu:
        yr = torch.relu(yr)
    yr.backward(dy.float())
    close(y, yr, what="bn fwd")
    close(xg.grad, xr.grad, rtol=3e-2, atol=3e-2, what="bn dx")
    close(gg, gr.grad, rtol=1e-2, atol=5e-2, what="bn dgamma")
    close(gbt, br.grad, rtol=1e-2, atol=5e-2, what="bn dbeta")
    if resid:
        close(rg.grad, rr.grad, what="bn dresid")
    n = N * H * W
    close(rm, 0.1 * mean.detach(), rtol=1e-3, atol=1e-3, what="running mean")
    close(rv, 0.9 + 0.1 * var.detach() * n / (n - 1), rtol=1e-3, atol=1e-3, what="running var")


@pytest.mark.parametrize("Cc", [64, 256, 2048, 200])
def test_bn_apply_dual(Cc):
    """bn_apply with a pre-BN residual normalised in the same sweep (ResNet downsample shortcut):
    relu(x*s + t + r*rs + rt) and its bit mask, vs fp32 torch on the same bf16 inputs."""
    M = 3 * 49 + 5
    x = rnd(M, Cc, seed=21)
    r = rnd(M, Cc, seed=22)
    s, t = torch.rand(Cc, device=DEV) + 0.5, torch.randn(Cc, device=DEV) * 0.1
    rs, rt = torch.rand(Cc, device=DEV) + 0.5, torch.randn(Cc, device=DEV) * 0.1
    y = torch.empty_like(x)
    mask = torch.zeros(-(-x.numel() // 32) * 4, dtype=torch.uint8, device=DEV)
    _C().bn_apply(x, s, t, r, y, Cc, True, mask, rs, rt)
    pre = x.float() * s + t + (r.float() * rs + rt)
    close(y, torch.relu(pre), rtol=1e-2, atol=1e-2, what="dual apply")
    # the bit mask (bn.hip relu_mask mode 3): element e = 8 v + i of 16-B vector v is bit i of byte v
    e = torch.arange(x.numel())
    bits = (mask.cpu().long()[e >> 3] >> (e & 7)) & 1
    ref = (pre.flatten().cpu() > 0).long()
    assert (bits != ref).float().mean().item() < 1e-3


@pytest.mark.parametrize("M,Cc", [(300007, 64), (100003, 512), (4099, 2048)])
def test_bn_sweeps_grid_stride(monkeypatch, M, Cc):
    """bn_apply (residual + bit mask) and bn_bwd_dx (modes 2 and 3, residual-gradient output) on row
    counts with a ragged last 2-row group per lane, vs fp32 torch on the same bf16 inputs."""
    x = rnd(M, Cc, seed=23)
    r = rnd(M, Cc, seed=24)
    dy = rnd(M, Cc, seed=25)
    s, t = torch.rand(Cc, device=DEV) + 0.5, torch.randn(Cc, device=DEV) * 0.1
    coef = torch.randn(3 * Cc, device=DEV)
    A, B, K = coef.view(3, Cc)
    y = torch.empty_like(x)
    mask = torch.zeros(-(-x.numel() // 32) * 4, dtype=torch.uint8, device=DEV)
    _C().bn_apply(x, s, t, r, y, Cc, True, mask)
    pre = x.float() * s + t + r.float()
    close(y, torch.relu(pre), rtol=1e-2, atol=1e-2, what="apply")
    e = torch.arange(x.numel(), device=DEV)
    bits = (mask.long()[e >> 3] >> (e & 7)) & 1
    assert (bits != (pre.flatten() > 0).long()).float().mean().item() < 1e-3
    dx, dres = torch.empty_like(x), torch.empty_like(x)
    _C().bn_bwd_dx(dy, x, mask, s, t, coef, dx, dres, Cc, 3)
    d = dy.float() * (bits.view(M, Cc) > 0)
    close(dres, d, rtol=1e-2, atol=1e-2, what="dx mode 3 dres")
    close(dx, A * d + B * x.float() + K, rtol=2e-2, atol=2e-2, what="dx mode 3")
    _C().bn_bwd_dx(dy, x, None, s, t, coef, dx, None, Cc, 2)
    d = dy.float() * ((x.float() * s + t) > 0)
    close(dx, A * d + B * x.float() + K, rtol=2e-2, atol=2e-2, what="dx mode 2")


# ----------------------------------------------------------------------------- pooling
@pytest.mark.parametrize("k,s,p,H", [(3, 2, 1, 16), (2, 2, 0, 24), (3, 2, 1, 15)])
def test_maxpool(k, s, p, H):
    from distributeddeeplearningspark_amd.ops.pool import max_pool2d

    x = rnd(2, H, H, 64, seed=19)
    xg = x.clone().requires_grad_(True)
    y = max_pool2d(xg, k, s, p)
    dy = rnd(*y.shape, seed=20)
    y.backward(dy)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.max_pool2d(xr, k, s, p)
    yr.backward(dy.float().permute(0, 3, 1, 2))
    close(y, yr.permute(0, 2, 3, 1), what="maxpool fwd")
    close(xg.grad, xr.grad.permute(0, 2, 3, 1), what="maxpool bwd")


def test_global_avgpool():
    from distributeddeeplearningspark_amd.ops.pool import global_avg_pool

    x = rnd(4, 7, 7, 2048, seed=21)
    xg = x.clone().requires_grad_(True)
    y = global_avg_pool(xg)
    dy = rnd(*y.shape, seed=22)
    y.backward(dy)
    close(y, x.float().mean((1, 2)), what="avgpool fwd")
    close(xg.grad, (dy.float() / 49).view(4, 1, 1, 2048).expand_as(xg), what="avgpool bwd")


# ----------------------------------------------------------------------------- loss
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_softmax_xent(dtype):
    from distributeddeeplearningspark_amd.ops.loss import softmax_cross_entropy

    B, K = 64, 1000
    logits = rnd(B, K, scale=3.0, dtype=dtype, seed=23)
    labels = torch.randint(0, K, (B,), device=DEV)
    lg = logits.clone().requires_grad_(True)
    loss = softmax_cross_entropy(lg, labels=labels)
    loss.backward()
    lr = logits.detach().float().clone().requires_grad_(True)
    ref = F.cross_entropy(lr, labels)
    ref.backward()
    assert abs(loss.item() - ref.item()) < 1e-3 * max(1.0, ref.item())
    close(lg.grad, lr.grad, rtol=2e-2, atol=1e-4, what="xent grad")
    probs = F.one_hot(labels, K).float()
    lg2 = logits.clone().requires_grad_(True)
    loss2 = softmax_cross_entropy(lg2, probs=probs)
    loss2.backward()
    assert abs(loss2.item() - ref.item()) < 1e-3 * max(1.0, ref.item())
    close(lg2.grad, lr.grad, rtol=2e-2, atol=1e-4, what="xent(probs) grad")


@pytest.mark.parametrize("form", ["sparse", "dense"])
def test_prob_xent_matches_fp32(form):
    """Keras CE on probabilities (a softmax OUTPUT layer, not fused into the loss): the HIP sweep
    (ops/loss.py prob_cross_entropy) vs the clipped fp32 formula, loss and d loss / d p, including
    probabilities below the clip (zero gradient) and an ignored label."""
    from distributeddeeplearningspark_amd.ops.loss import prob_cross_entropy

    B, K = 37, 10
    p = torch.softmax(rnd(B, K, scale=6.0, dtype=torch.float32, seed=41), dim=-1)
    p[0, 3] = 1e-9  # below the clip
    labels = torch.randint(0, K, (B,), device=DEV)
    labels[0] = 3
    y = F.one_hot(labels, K).float()
    pg = p.clone().requires_grad_(True)
    loss = prob_cross_entropy(pg, labels=labels) if form == "sparse" else prob_cross_entropy(pg, target=y)
    loss.backward()
    pr = p.clone().requires_grad_(True)
    ref = -(y * torch.log(pr.clamp(1e-7, 1 - 1e-7))).sum(-1).mean()
    ref.backward()
    assert abs(loss.item() - ref.item()) < 1e-5 * max(1.0, abs(ref.item())), (loss.item(), ref.item())
    close(pg.grad, pr.grad, rtol=1e-5, atol=1e-6, what=f"prob xent grad ({form})")
    assert pg.grad[0, 3].item() == 0.0
    if form == "sparse":  # ignore_index rows contribute neither loss nor gradient
        lab2 = labels.clone()
        lab2[1] = -100
        pg2 = p.clone().requires_grad_(True)
        l2 = prob_cross_entropy(pg2, labels=lab2)
        l2.backward()
        assert torch.all(pg2.grad[1] == 0)
        keep = torch.ones(B, device=DEV)
        keep[1] = 0
        ref2 = (-(y * torch.log(p.clamp(1e-7, 1 - 1e-7))).sum(-1) * keep).sum() / B
        assert abs(l2.item() - ref2.item()) < 1e-5


def test_softmax_xent_padded_vocab():
    """The MLM decoder's call: bf16 logits rows padded to 30,528 columns, the first 30,522 are the
    vocabulary (16-B vector passes + a 2-column scalar tail); dlogits' padding columns come back 0."""
    B, V, Vp = 96, 30522, 30528
    full = rnd(B, Vp, scale=4.0, seed=31)
    labels = torch.randint(0, V, (B,), device=DEV)
    labels[5] = -100  # ignored row
    loss_rows = torch.empty(B, device=DEV)
    dl = torch.full((B, Vp), 7.0, dtype=torch.bfloat16, device=DEV)
    n_valid = int((labels != -100).sum())
    _C().softmax_xent(full[:, :V], labels, None, loss_rows, dl[:, :V], 1.0 / n_valid, 0.0, -100)
    lr = full[:, :V].float().clone().requires_grad_(True)
    ref = F.cross_entropy(lr, labels, ignore_index=-100, reduction="sum") / n_valid
    ref.backward()
    assert abs(loss_rows.sum().item() / n_valid - ref.item()) < 1e-3 * max(1.0, ref.item())
    close(dl[:, :V], lr.grad, rtol=2e-2, atol=1e-6, what="padded-vocab xent grad")
    assert torch.all(dl[:, V:] == 0)
    assert torch.all(dl[5] == 0)


# ----------------------------------------------------------------------------- optimizers
@pytest.mark.parametrize("kind", ["sgd", "sgd_nesterov", "adam", "adamw", "adam_keras", "adagrad", "rmsprop"])
def test_optimizers(kind):
    from distributeddeeplearningspark_amd.ops import optim as O

    n = 4096 + 64
    w0 = torch.randn(n)
    g = torch.randn(n)
    outs = {}
    for dev in ("cpu", DEV):
        w = w0.clone().to(dev)
        gd = g.to(dev)
        s1, s2 = torch.zeros(n, device=dev), torch.zeros(n, device=dev)
        w16 = torch.empty(n, dtype=torch.bfloat16, device=dev) if dev != "cpu" else None
        for step in range(1, 4):
            if kind.startswith("sgd"):
                O.sgd_(w, gd, s1, w16, lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=kind == "sgd_nesterov",
                       grad_scale=0.5)
            elif kind == "adam":
                O.adam_(w, gd, s1, s2, w16, lr=1e-3, weight_decay=1e-2, step=step)
            elif kind == "adamw":
                O.adam_(w, gd, s1, s2, w16, lr=1e-3, weight_decay=1e-2, decoupled=True, step=step)
            elif kind == "adam_keras":
                O.adam_(w, gd, s1, s2, w16, lr=1e-3, eps=1e-7, keras_eps=True, step=step)
            elif kind == "adagrad":
                O.adagrad_(w, gd, s1, w16, lr=1e-2)
            else:
                O.rmsprop_(w, gd, s1, w16, lr=1e-3)
        outs[dev] = (w.cpu(), None if w16 is None else w16.float().cpu())
    close(outs[DEV][0], outs["cpu"][0], rtol=1e-5, atol=1e-6, what=f"{kind} master")
    close(outs[DEV][1], outs["cpu"][0], rtol=1e-2, atol=1e-2, what=f"{kind} bf16 copy")


# ----------------------------------------------------------------------------- misc
def test_normalize_u8_and_casts():
    from distributeddeeplearningspark_amd.data.ingest import DeviceFeeder

    f = DeviceFeeder(DEV)
    # 4-pixel RGB kernel (pixel count % 4 == 0, incl. an ImageNet-size batch) and the per-element kernel
    for shape in ((2, 8, 8, 3), (1, 5, 5, 3), (16, 224, 224, 3)):
        x = torch.randint(0, 256, shape, dtype=torch.uint8, device=DEV)
        y = f.normalize(x)
        ref = (x.float() - f.mean) * f.invstd
        close(y, ref, what=f"normalize_u8 {shape}")
        assert torch.equal(y, ref.to(torch.bfloat16)), shape  # same fp32 formula, RNE to bf16
    a = torch.randn(1003, device=DEV)
    b = torch.empty(1003, dtype=torch.bfloat16, device=DEV)
    _C().cast_f32_bf16(a, b)
    assert torch.equal(b, a.to(torch.bfloat16))


def test_linear_layer_odd_sizes():
    from distributeddeeplearningspark_amd.ops.linear import linear

    for (M, K, N) in [(16, 4608, 225), (16, 225, 10), (32, 128, 1)]:
        x = rnd(M, K, seed=24)
        w = rnd(N, K, scale=1 / math.sqrt(K), seed=25)
        b = torch.randn(N, device=DEV)
        gw, gb = torch.zeros(N, K, device=DEV), torch.zeros(N, device=DEV)
        xg = x.clone().requires_grad_(True)
        y = linear(xg, w.clone().requires_grad_(True), b, relu=True, grad_w=gw, grad_b=gb)
        dy = rnd(M, N, seed=26)
        y.backward(dy)
        xr, wr, br = x.float().requires_grad_(True), w.float().requires_grad_(True), b.clone().requires_grad_(True)
        yr = torch.relu(xr @ wr.T + br)
        yr.backward(dy.float())
        close(y, yr, what=f"linear fwd {(M, K, N)}")
        close(xg.grad, xr.grad, what=f"linear dgrad {(M, K, N)}")
        close(gw, wr.grad, rtol=1e-2, atol=1e-2, what=f"linear wgrad {(M, K, N)}")
        close(gb, br.grad, rtol=1e-2, atol=1e-2, what=f"linear bgrad {(M, K, N)}")


def test_resnet50_step_matches_reference():
    """Small ResNet-50 (64x64 input): GPU bf16 loss / gradient norm inside the fp32 CPU path's own spread.

    At random init this network's gradient norm moves by percents under input perturbations far below
    bf16 resolution: on the CPU in fp32, x (1 + 2^-9 n) gives 555.6 / 564.7 / 571.7 against 580.5
    unperturbed, and the HIP path lands at 560.6 / 563.8 on the base input and 580.4 / 588.0 / 586.9 on
    perturbed ones (profiles/r5/gradnorm_spread.txt; per-layer ratios: profiles/r5/gradnorm_layers.txt).
    The round-4 "undershoot" (553-572 vs 580) was the unperturbed fp32 point sitting high in that spread,
    not a HIP bias (the losses spread the same way: fp32 2.30-2.51, HIP 2.38-2.59).  So the reference is the
    fp32 ensemble — the base input and three 2^-9 perturbations — and the HIP loss and norm must lie inside its
    envelope widened by 4 % (round 4 had widened a band around the single unperturbed point to 8 %)."""
    from distributeddeeplearningspark_amd.models import ResNet50

    import os

    torch.manual_seed(0)
    x = torch.randn(16, 64, 64, 3)
    y = torch.randint(0, 10, (16,))

    def step(dev, xin, ref=False):
        old = os.environ.get("DDL_BACKEND")
        if ref:
            os.environ["DDL_BACKEND"] = "torch"  # same bf16 model through PyTorch/MIOpen ops
        try:
            m = ResNet50(input_shape=(64, 64, 3), num_classes=10)
            m.compile("sgd", "sparse_categorical_crossentropy")
            m.place(dev, seed=3)
            loss = m.backward_step(m.to_input(xin), m.to_target(y))
            return float(loss.detach()), m.arena.grad.norm().item()
        finally:
            if old is None:
                os.environ.pop("DDL_BACKEND", None)
            else:
                os.environ["DDL_BACKEND"] = old

    cpu = [step("cpu", x)]
    for k in range(3):
        g = torch.Generator().manual_seed(100 + k)
        cpu.append(step("cpu", x * (1 + 2.0 ** -9 * torch.randn(x.shape, generator=g))))
    lc = sum(c[0] for c in cpu) / len(cpu)
    gc = sum(c[1] for c in cpu) / len(cpu)
    lh, gh = step(DEV, x)
    ll, gl = step(DEV, x, ref=True)
    res = {"cpu_fp32_ensemble": cpu, "hip": (lh, gh), "torch_bf16": (ll, gl)}
    print("ResNet-50 step (loss, grad norm):", res)

    def inside(v, i, margin):  # inside the fp32 ensemble's envelope, widened by margin x its mean
        lo, hi, mean = min(c[i] for c in cpu), max(c[i] for c in cpu), sum(c[i] for c in cpu) / len(cpu)
        return lo - margin * mean <= v <= hi + margin * mean

    assert inside(lh, 0, 0.04) and inside(gh, 1, 0.04), res
    assert abs(ll - lc) < 0.12 * max(1.0, abs(lc)) and abs(gl - gc) < 0.08 * gc, res


def test_fused_bottleneck_matches_composed_ops():
    """ops/fused_blocks.py (one autograd node per block) vs the per-op autograd graph.

    A one-block ResNet (stem + one bottleneck with projection shortcut): the full-depth
    random-init ResNet-50 at a tiny batch is chaotic (1-ulp bf16 flips from atomic-order
    differences in the BN statistics move its loss by percents), so the comparison is made
    where it is well conditioned."""
    import os

    from distributeddeeplearningspark_amd.models import resnet as RN
    from distributeddeeplearningspark_amd.models.resnet import ResNet

    torch.manual_seed(1)
    x = torch.randn(16, 32, 32, 3)
    y = torch.randint(0, 10, (16,))
    res = {}
    for fused, dev in (("1", DEV), ("0", DEV), ("0", "cpu")):
        old = RN.FUSED_BLOCKS
        RN.FUSED_BLOCKS = fused == "1"
        try:
            m = ResNet(blocks=(2,), input_shape=(32, 32, 3), num_classes=10)
            m.compile("sgd", "sparse_categorical_crossentropy")
            m.place(dev, seed=5)
            loss = m.backward_step(m.to_input(x), m.to_target(y))
            res[fused + dev] = (float(loss.detach()), m.arena.to_canonical(m.arena.grad.detach()).float().cpu().clone())
        finally:
            RN.FUSED_BLOCKS = old
    l1, l0, lc = res["1" + DEV][0], res["0" + DEV][0], res["0cpu"][0]
    assert abs(l1 - l0) < 1e-2 * max(1.0, abs(l0)), (l1, l0)
    # the fused node applies the downsample BN inside the block-output sweep (the shortcut is never
    # rounded to bf16), so it differs from the composed bf16 graph by that rounding; both must sit
    # as close to the fp32 CPU gradients (bf16 noise through the BN backward: ~5-8 % per layer)
    g1, g0, gc = res["1" + DEV][1], res["0" + DEV][1], res["0cpu"][1]
    e1, e0 = ((g1 - gc).norm() / gc.norm()).item(), ((g0 - gc).norm() / gc.norm()).item()
    assert e1 < 1.25 * e0 + 1e-2 and e1 < 0.1, (e1, e0)
    assert ((g1 - g0).norm() / g0.norm()).item() < 6e-2


@pytest.mark.parametrize("kind", ["adam", "adamw", "adam_keras"])
def test_adam_paired_slot_loop(kind):
    """n = 2 x (4096 x 256 grid) x 4 plus an odd number of float4 slots (flat arenas are
    multiples of 4): the two-float4-per-lane loop of the Adam kernel and its single-slot tail
    both run (the small test above only reaches the tail); master weights, moments and the bf16
    compute copy against the CPU reference."""
    from distributeddeeplearningspark_amd.ops import optim as O

    n = 2 * 4096 * 256 * 4 + 4 * 5
    gen = torch.Generator().manual_seed(21)
    w0, g = torch.randn(n, generator=gen), torch.randn(n, generator=gen)
    outs = {}
    for dev in ("cpu", DEV):
        w, gd = w0.clone().to(dev), g.to(dev)
        m, v = torch.zeros(n, device=dev), torch.zeros(n, device=dev)
        w16 = torch.empty(n, dtype=torch.bfloat16, device=dev) if dev != "cpu" else None
        for step in range(1, 3):
            if kind == "adam":
                O.adam_(w, gd, m, v, w16, lr=1e-3, weight_decay=1e-2, step=step)
            elif kind == "adamw":
                O.adam_(w, gd, m, v, w16, lr=1e-3, weight_decay=1e-2, decoupled=True, step=step)
            else:
                O.adam_(w, gd, m, v, w16, lr=1e-3, eps=1e-7, keras_eps=True, step=step)
        outs[dev] = (w.cpu(), m.cpu(), v.cpu(), None if w16 is None else w16.float().cpu())
    close(outs[DEV][0], outs["cpu"][0], rtol=1e-5, atol=1e-6, what=f"{kind} master")
    close(outs[DEV][1], outs["cpu"][1], rtol=1e-5, atol=1e-6, what=f"{kind} m")
    close(outs[DEV][2], outs["cpu"][2], rtol=1e-5, atol=1e-6, what=f"{kind} v")
    close(outs[DEV][3], outs["cpu"][0], rtol=1e-2, atol=1e-2, what=f"{kind} bf16 copy")
    # every index of the tail was written (a skipped element would keep w0)
    assert not torch.equal(outs[DEV][0][-20:], w0[-20:])


def test_resnet_per_layer_gradients_match_fp32_cpu():
    """Per-parameter-tensor gradients of a 4-bottleneck ResNet (one block per stage, batch 32,
    32x32) from the same weights on three paths: fp32 CPU (reference), the bf16 HIP kernels,
    and the same bf16 model through PyTorch/MIOpen (``DDL_BACKEND=torch``).  bf16 rounding of
    the activations alone costs the early layers some gradient direction (cosine ~0.93-0.95 vs
    fp32 on BOTH bf16 paths), so each layer's HIP gradient must be at least as close to fp32 as
    the library's (cosine within 0.03 of it — measured: HIP 0.92-0.95 vs library 0.94-0.96 on the
    BN affine gradients, the conv kernels within 0.01 — above an absolute floor of 0.85, norm
    within 8 % (BN gamma/beta sums run 3-5 % off fp32 from atomic-order noise)): a wrong
    term in any single backward kernel (BN, ReLU mask, residual, dgrad/wgrad) drops that layer's
    cosine far below the library path instead of averaging away in a whole-model norm."""
    import os

    from distributeddeeplearningspark_amd.models.resnet import ResNet

    torch.manual_seed(4)
    x = torch.randn(32, 32, 32, 3)
    y = torch.randint(0, 10, (32,))
    grads, losses = {}, {}
    for name, dev, lib in (("cpu", "cpu", False), ("hip", DEV, False), ("lib", DEV, True)):
        old = os.environ.get("DDL_BACKEND")
        if lib:
            os.environ["DDL_BACKEND"] = "torch"
        try:
            m = ResNet((1, 1, 1, 1), num_classes=10, input_shape=(32, 32, 3), name="rn_small")
            m.compile("sgd", "sparse_categorical_crossentropy")
            m.place(dev, seed=5)
            loss = m.backward_step(m.to_input(x), m.to_target(y))
            losses[name] = float(loss.detach())
            grads[name] = {p.name: p.grad.detach().float().cpu().reshape(-1).clone()
                           for p in m.arena.params if p.trainable}
        finally:
            if old is None:
                os.environ.pop("DDL_BACKEND", None)
            else:
                os.environ["DDL_BACKEND"] = old
    assert abs(losses["hip"] - losses["cpu"]) < 0.02 * abs(losses["cpu"]), losses
    bad, worst = [], 1.0
    for pname, gc in grads["cpu"].items():
        nc = gc.norm().item()
        if nc < 1e-6:
            continue
        cos = {k: torch.nn.functional.cosine_similarity(grads[k][pname], gc, dim=0).item() for k in ("hip", "lib")}
        rel = {k: abs(grads[k][pname].norm().item() - nc) / nc for k in ("hip", "lib")}
        worst = min(worst, cos["hip"])
        if cos["hip"] < min(cos["lib"] - 0.03, 0.995) or cos["hip"] < 0.85 or rel["hip"] > max(0.08, rel["lib"] + 0.03):
            bad.append((pname, round(cos["hip"], 4), round(cos["lib"], 4), round(rel["hip"], 4), round(rel["lib"], 4)))
    assert not bad, f"(layer, cos hip, cos lib, norm err hip, norm err lib): {bad}"


@pytest.mark.parametrize("N,H,W,Ci,Co", [(3, 56, 56, 64, 64), (2, 28, 28, 128, 128), (5, 14, 14, 256, 256),
                                         (9, 7, 7, 512, 512), (2, 20, 12, 64, 192), (4, 9, 9, 128, 64)])
@pytest.mark.parametrize("bias_relu", [False, True])
def test_conv3x3_halo_kernel(N, H, W, Ci, Co, bias_relu, monkeypatch):
    """3x3 stride-1 halo kernel (csrc/kernels/conv3x3.hip) vs fp32 PyTorch: whole-row tiles of
    one image (56/28/20 wide), whole images per tile with a partial last group of images (N=9 at
    7x7, N=5 at 14x14), 64- and 128-channel output tiles, bias+ReLU and the fused BN statistics."""
    from distributeddeeplearningspark_amd.ops import conv as CV
    from distributeddeeplearningspark_amd.ops import gemm as G

    g = CV.geometry(N, H, W, Ci, Co, 3, 3, (1, 1), (1, 1), (1, 1))
    if Ci == 64 and Co == 64:  # one 64-channel chunk: conv.halo3_ok routes it to the implicit GEMM
        assert not CV.halo3_ok(g)
    else:
        assert CV.halo3_ok(g)
    x = rnd(N, H, W, Ci, seed=1)
    w = rnd(Co, 3, 3, Ci, scale=0.05, seed=2)
    b = torch.randn(Co, device=DEV) * 0.1 if bias_relu else None
    st = torch.zeros((32, 2, Co), dtype=torch.float32, device=DEV)
    y = CV.conv_fwd_native(x, w, g, bias=b, relu=bias_relu, stats=st)
    ref = CV.conv_ref(x.float(), w.float(), b, (1, 1), (1, 1), (1, 1), relu=bias_relu)
    close(y, ref, what="halo conv")
    yf = y.float().reshape(-1, Co)
    close(st.sum(0)[0], yf.sum(0), rtol=1e-3, atol=1e-1, what="halo stats sum")
    close(st.sum(0)[1], (yf * yf).sum(0), rtol=1e-3, atol=1e-1, what="halo stats sumsq")
    # the implicit-GEMM kernel on the same problem agrees too (same bf16 rounding of the output)
    y2 = torch.empty_like(y)
    G.gemm(x, w, y2.view(g.M, Co), g.M, Co, 9 * Ci, G.KC_GATHER, G.KC, 0, 9 * Ci, Co, G.EPI_BF16, bias=b,
           relu=bias_relu, geom=g.fwd_geom)
    close(y, y2, rtol=1e-2, atol=1e-2, what="halo vs implicit GEMM")


@pytest.mark.parametrize("M,N,K,resid,mode", [(16384, 256, 64, True, 3), (20000, 512, 128, True, 3),
                                              (16384, 1024, 256, False, 3), (32768, 64, 256, False, 2),
                                              (16384, 256, 64, False, 2), (16384, 128, 128, False, 2)])
def test_stream_dgrad_fused_bn_backward_reduce(M, N, K, resid, mode):
    """linear_dgrad on the streaming kernel with ``bnr``: the output equals the plain launch, and the
    workspace holds sum_m d*relu and sum_m d*relu*(x - mean) of the STORED output (fp64 reference),
    with relu the mode-3 bit mask or (mode 2) x * scale + shift > 0 — the partial sums bn_bwd_reduce
    would have produced.  (32768, 64, 256): ResNet-50 stage 1's conv3 data-gradient feeding bn2."""
    from distributeddeeplearningspark_amd.ops import gemm as G
    from distributeddeeplearningspark_amd.ops.norm import SHARDS

    gen = torch.Generator().manual_seed(M + N)
    dy = torch.randn(M, K, generator=gen).to(DEV, torch.bfloat16)
    w = (torch.randn(K, N, generator=gen) / K ** 0.5).to(DEV, torch.bfloat16)
    r = torch.randn(M, N, generator=gen).to(DEV, torch.bfloat16) if resid else None
    x = torch.randn(M, N, generator=gen).to(DEV, torch.bfloat16)
    keep = torch.rand(M, N, generator=gen) > 0.4
    bits = (keep.reshape(-1, 8).to(torch.uint8) << torch.arange(8, dtype=torch.uint8)).sum(1, dtype=torch.uint8)
    mask = bits.to(DEV)
    mean = torch.randn(N, generator=gen).to(DEV)
    assert G.use_stream(M, N, K, G.KC, G.RC, G.EPI_BF16, K, N, resid=r, ldr=N if resid else 0)
    ws = torch.zeros((SHARDS, 2, N), dtype=torch.float32, device=DEV)
    bnr = {"x": x, "mask": mask, "mean": mean, "ws": ws}
    if mode == 2:
        scale = (torch.rand(N, generator=gen) + 0.5).to(DEV)
        shift = torch.randn(N, generator=gen).to(DEV) * 0.5
        bnr = {"x": x, "scale": scale, "shift": shift, "mean": mean, "ws": ws}
        keep = (x.float() * scale + shift > 0).cpu()
    out = G.linear_dgrad(dy, w, resid=r, bnr=bnr)
    assert bnr.get("done")
    ref_out = G.linear_dgrad(dy, w, resid=r)
    assert torch.equal(out, ref_out)
    d = out.double().cpu() * keep.double()
    s1 = d.sum(0)
    s2 = (d * (x.double().cpu() - mean.double().cpu())).sum(0)
    got = ws.double().cpu().sum(0)
    close(got[0], s1, rtol=1e-4, atol=1e-2 * s1.abs().mean().item(), what="sum d")
    close(got[1], s2, rtol=1e-4, atol=1e-2 * s2.abs().mean().item(), what="sum d (x - mean)")


def _bnr_reference(out, x, mean, keep):
    d = out.double().cpu().reshape(-1, out.shape[-1]) * keep.double()
    return d.sum(0), (d * (x.double().cpu().reshape(d.shape) - mean.double().cpu())).sum(0)


@pytest.mark.parametrize("M,N,K,mode", [(8192, 512, 128, 2), (8192, 512, 128, 3), (2048, 256, 192, 2)])
def test_dma_dgrad_fused_bn_backward_reduce(M, N, K, mode):
    """linear_dgrad on the LDS-DMA GEMM (transposed-weight KC x KC path for M >= 4096, KC x RC below)
    with ``bnr``: EPI_BF16_BNR stores the same output as the plain launch and accumulates the BN-backward
    partial sums with the mode-2 (x * scale + shift > 0) or mode-3 (bit) ReLU mask."""
    from distributeddeeplearningspark_amd.ops import gemm as G
    from distributeddeeplearningspark_amd.ops.norm import SHARDS

    gen = torch.Generator().manual_seed(M + N + mode)
    dy = torch.randn(M, N, generator=gen).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, generator=gen) / N ** 0.5).to(DEV, torch.bfloat16)
    x = torch.randn(M, K, generator=gen).to(DEV, torch.bfloat16)
    mean = torch.randn(K, generator=gen).to(DEV)
    ws = torch.zeros((SHARDS, 2, K), dtype=torch.float32, device=DEV)
    bnr = {"x": x, "mean": mean, "ws": ws}
    if mode == 2:
        scale = (torch.rand(K, generator=gen) + 0.5).to(DEV)
        shift = torch.randn(K, generator=gen).to(DEV) * 0.5
        bnr.update(scale=scale, shift=shift)
        keep = (x.float() * scale + shift > 0).cpu()
    else:
        keep = torch.rand(M, K, generator=gen) > 0.4
        bnr["mask"] = (keep.reshape(-1, 8).to(torch.uint8) << torch.arange(8, dtype=torch.uint8)).sum(
            1, dtype=torch.uint8).to(DEV)
    assert not G.use_stream(M, K, N, G.KC, G.RC, G.EPI_BF16, N, K)
    out = G.linear_dgrad(dy, w, bnr=bnr)
    assert bnr.get("done")
    assert torch.equal(out, G.linear_dgrad(dy, w))
    s1, s2 = _bnr_reference(out, x, mean, keep)
    got = ws.double().cpu().sum(0)
    close(got[0], s1, rtol=1e-4, atol=1e-2 * s1.abs().mean().item(), what="sum d")
    close(got[1], s2, rtol=1e-4, atol=1e-2 * s2.abs().mean().item(), what="sum d (x - mean)")


@pytest.mark.parametrize("N,H,C", [(96, 14, 128), (160, 16, 64)])
def test_conv_dgrad_fused_bn_backward_reduce(monkeypatch, N, H, C):
    """A stride-1 3x3 data-gradient run as a forward conv (halo kernel at 128 channels, the gathered
    implicit GEMM at 64) with a mode-2 ``bnr``: same dx as without, and the BN-backward partial sums."""
    from distributeddeeplearningspark_amd.ops import conv as CV
    from distributeddeeplearningspark_amd.ops.norm import SHARDS

    g = CV.geometry(N, H, H, C, C, 3, 3, (1, 1), (1, 1), (1, 1))
    assert CV.halo3_ok(g) == (C >= 128) and not CV.splitk_fwd_ok(g)  # (small grids take the split-K path)
    gen = torch.Generator().manual_seed(H * C)
    dy = torch.randn(N, H, H, C, generator=gen).to(DEV, torch.bfloat16)
    w = (torch.randn(C, 3, 3, C, generator=gen) * 0.05).to(DEV, torch.bfloat16)
    x = torch.randn(N, H, H, C, generator=gen).to(DEV, torch.bfloat16)
    mean = torch.randn(C, generator=gen).to(DEV) * 0.1
    scale = (torch.rand(C, generator=gen) + 0.5).to(DEV)
    shift = torch.randn(C, generator=gen).to(DEV) * 0.5
    ws = torch.zeros((SHARDS, 2, C), dtype=torch.float32, device=DEV)
    bnr = {"x": x, "scale": scale, "shift": shift, "mean": mean, "ws": ws}
    dx = CV.conv_dgrad_native(dy, w, g, bnr=bnr)
    assert bnr.get("done")
    assert torch.equal(dx, CV.conv_dgrad_native(dy, w, g))
    keep = (x.float() * scale + shift > 0).cpu().reshape(-1, C)
    s1, s2 = _bnr_reference(dx, x, mean, keep)
    got = ws.double().cpu().sum(0)
    close(got[0], s1, rtol=1e-4, atol=1e-2 * s1.abs().mean().item(), what="sum d")
    close(got[1], s2, rtol=1e-4, atol=1e-2 * s2.abs().mean().item(), what="sum d (x - mean)")


def test_bottleneck_inner_fused_bn_reduce_matches_unfused(monkeypatch):
    """bn1 / bn2 backward reduces fused into the conv2 / conv3 data-gradient epilogues (stage 1: the 64-channel
    gathered conv2 dgrad; stage 2: the transposed-weight conv3 dgrad): fewer reduce sweeps, same gradients.
    (At this batch the stage-1 conv2 dgrads take the split-K path and stage 1's conv3 dgrads the streaming
    kernel, neither of which fuses a mode-2 reduce: the two stage-2 conv3 dgrads do.)  Gradients are held
    to the unfused path's own run-to-run spread (tests/noise.py: BN-statistics atomics + bf16 rounding)."""
    from noise import assert_scalar_within_noise, assert_within_noise

    from distributeddeeplearningspark_amd.models.resnet import ResNet
    from distributeddeeplearningspark_amd.ops import fused_blocks as FB

    torch.manual_seed(4)
    x = torch.randn(64, 64, 64, 3)
    y = torch.randint(0, 10, (64,))
    out = []
    for fuse in (False, True, False):
        monkeypatch.setattr(FB, "_FUSE_BNR_INNER", fuse)
        m = ResNet(blocks=(2, 2), input_shape=(64, 64, 3), num_classes=10)
        m.compile("sgd", "sparse_categorical_crossentropy")
        m.place(DEV, seed=5)
        xd, yd = m.to_input(x), m.to_target(y)
        m.backward_step(xd, yd)
        from torch.profiler import ProfilerActivity, profile

        torch.cuda.synchronize()
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            loss = m.backward_step(xd, yd)
            torch.cuda.synchronize()
        n_reduce = sum(1 for e in prof.events() if "bn_bwd_reduce" in e.name)
        out.append((float(loss.detach()), m.arena.to_canonical(m.arena.grad.detach()).float().cpu().clone(), n_reduce))
    (l0, g0, r0), (l1, g1, r1), (l0b, g0b, _) = out
    assert r1 <= r0 - 2, (r1, r0)
    # the loss is the FORWARD's (both variants run the same forward kernels): its spread is the forward's own
    # BN-statistics noise, amplified by bf16 through the blocks (measured up to 5.6e-3 relative after four
    # blocks, tests/noise.py) — two reference runs under-sample it, hence the 1e-3 relative floor
    assert_scalar_within_noise(l1, l0, l0b, floor=1e-3)
    assert_within_noise(g1, g0, g0b, floor=2e-3, what="arena gradients")


@pytest.mark.parametrize("M,N,K,rsub", [(12544, 512, 2048, False), (8192, 256, 1024, True)])
def test_dma_dgrad_fused_bn_reduce_with_residual(M, N, K, rsub):
    """linear_dgrad on the LDS-DMA GEMM with a residual AND ``bnr`` (mode 3): the identity shortcut's masked
    gradient (resid + resid_mask) or the stride-2 shortcut's half-resolution gradient (rsub) added in the
    EPI_BF16_BNR epilogue — the same output as the full epilogue, and the reduce of the stored sum
    (ResNet-50 stage 4's conv1 data-gradients and the stage-3 -> 4 boundary)."""
    from distributeddeeplearningspark_amd.ops import gemm as G
    from distributeddeeplearningspark_amd.ops.norm import SHARDS

    gen = torch.Generator().manual_seed(M + K)
    dy = torch.randn(M, N, generator=gen).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, generator=gen) / N ** 0.5).to(DEV, torch.bfloat16)
    x = torch.randn(M, K, generator=gen).to(DEV, torch.bfloat16)
    mean = torch.randn(K, generator=gen).to(DEV)
    keep = torch.rand(M, K, generator=gen) > 0.4
    mbits = (keep.reshape(-1, 8).to(torch.uint8) << torch.arange(8, dtype=torch.uint8)).sum(1, dtype=torch.uint8)
    if rsub:  # rows = [M / 64][8][8] grid, residual on its [4][4] even subgrid
        hw = 8
        r = torch.randn(M // 4, K, generator=gen).to(DEV, torch.bfloat16)
        kw = dict(resid=r, rsub=(hw, hw))
    else:
        r = torch.randn(M, K, generator=gen).to(DEV, torch.bfloat16)
        rk = torch.rand(M, K, generator=gen) > 0.5
        rmask = (rk.reshape(-1, 8).to(torch.uint8) << torch.arange(8, dtype=torch.uint8)).sum(1, dtype=torch.uint8)
        kw = dict(resid=r, resid_mask=rmask.to(DEV))
    assert not G.use_stream(M, K, N, G.KC, G.RC, G.EPI_BF16, N, K, resid=r, ldr=K)
    ws = torch.zeros((SHARDS, 2, K), dtype=torch.float32, device=DEV)
    bnr = {"x": x, "mask": mbits.to(DEV), "mean": mean, "ws": ws}
    out = G.linear_dgrad(dy, w, bnr=bnr, **kw)
    assert bnr.get("done")
    assert torch.equal(out, G.linear_dgrad(dy, w, **kw))
    s1, s2 = _bnr_reference(out, x, mean, keep)
    got = ws.double().cpu().sum(0)
    close(got[0], s1, rtol=1e-4, atol=1e-2 * s1.abs().mean().item(), what="sum d")
    close(got[1], s2, rtol=1e-4, atol=1e-2 * s2.abs().mean().item(), what="sum d (x - mean)")


@pytest.mark.parametrize("N,H,C,k", [(16, 112, 64, 3), (8, 57, 32, 3), (32, 32, 64, 2), (64, 4, 512, 2), (8, 16, 128, 2)])
def test_stem_pool_bn_backward_fused(N, H, C, k):
    """pool3s2_bn_bwd: the BN's reduce and dx sweeps computed through the max pool's gather (pooled gradient
    + argmax bytes) — the stem's 3x3 / 2 / pad-1 pool (k = 3) or a VGG block's 2x2 / 2 pool (k = 2) — match
    maxpool_bwd -> bn_bwd_reduce -> bn_bwd_dx (mode 2) on the materialised pool gradient: partial sums to
    fp32 rounding, dx to bf16 rounding."""
    from distributeddeeplearningspark_amd.ops._native import C as NC
    from distributeddeeplearningspark_amd.ops.norm import partials_workspace

    gen = torch.Generator().manual_seed(N * H + C)
    x = torch.randn(N, H, H, C, generator=gen).to(DEV, torch.bfloat16)
    scale = (torch.rand(C, generator=gen) + 0.5).to(DEV)
    shift = (torch.randn(C, generator=gen) * 0.5).to(DEV)
    mean = (torch.randn(C, generator=gen) * 0.1).to(DEV)
    p = 1 if k == 3 else 0
    Ho = (H + 2 * p - k) // 2 + 1
    y = torch.empty(N, Ho, Ho, C, dtype=torch.bfloat16, device=DEV)
    am = torch.empty(N, Ho, Ho, C, dtype=torch.uint8, device=DEV)
    NC().maxpool_fwd(x, y, am, k, k, 2, 2, p, p, scale, shift)
    dy = torch.randn(N, Ho, Ho, C, generator=gen).to(DEV, torch.bfloat16)
    d = torch.empty_like(x)
    NC().maxpool_bwd(dy, am, d, k, k, 2, 2, p, p)
    M = N * H * H
    ws_ref = partials_workspace(M, C, DEV)
    NC().bn_bwd_reduce(d, x, None, scale, shift, mean, ws_ref, C, 2)
    ws = torch.empty((1024, 2, C), dtype=torch.float32, device=DEV)
    assert NC().pool3s2_bn_bwd_ok(N, H, H, C, Ho, Ho, k)
    NC().pool3s2_bn_bwd(dy, am, x, scale, shift, mean, ws, None, k)
    ref, got = ws_ref.double().sum(0).cpu(), ws.double().sum(0).cpu()
    close(got[0], ref[0], rtol=1e-4, atol=1e-4 * ref[0].abs().mean().item(), what="sum d'")
    close(got[1], ref[1], rtol=1e-4, atol=1e-4 * ref[1].abs().mean().item(), what="sum d' (x - mean)")
    coef = torch.randn(3 * C, generator=gen).to(DEV)
    dx_ref = torch.empty_like(x)
    NC().bn_bwd_dx(d, x, None, scale, shift, coef, dx_ref, None, C, 2)
    dx = torch.empty_like(x)
    NC().pool3s2_bn_bwd(dy, am, x, scale, shift, mean, coef, dx, k)
    close(dx.float(), dx_ref.float(), rtol=1e-2, atol=1e-2, what="dx")


def test_bn_bwd_dx_fused_second_reduce():
    """bn_bwd_dx_red: the dx sweep of a mode-3 BN (bit mask) also writes the reduce partials of a second
    BN fed by the masked gradient (ResNet downsample BN): dx equals bn_bwd_dx's, and the partial rows sum
    to bn_bwd_reduce's result on (dy, x2, mask) — the fp64 reference of sum d, sum d (x2 - mean2)."""
    from distributeddeeplearningspark_amd.ops._native import C as NC
    from distributeddeeplearningspark_amd.ops.norm import partials_workspace

    for M, Cc in ((50176, 256), (12544, 2048), (4000, 192)):
        gen = torch.Generator().manual_seed(M + Cc)
        dy = torch.randn(M, Cc, generator=gen).to(DEV, torch.bfloat16)
        x = torch.randn(M, Cc, generator=gen).to(DEV, torch.bfloat16)
        x2 = torch.randn(M, Cc, generator=gen).to(DEV, torch.bfloat16)
        keep = torch.rand(M, Cc, generator=gen) > 0.4
        mask = (keep.reshape(-1, 8).to(torch.uint8) << torch.arange(8, dtype=torch.uint8)).sum(
            1, dtype=torch.uint8).to(DEV)
        coef = torch.randn(3 * Cc, generator=gen).to(DEV)
        mean2 = (torch.randn(Cc, generator=gen) * 0.1).to(DEV)
        dx_ref = torch.empty_like(dy)
        dres = torch.empty_like(dy)
        NC().bn_bwd_dx(dy, x, mask, None, None, coef, dx_ref, dres, Cc, 3)
        dx = torch.empty_like(dy)
        ws2 = partials_workspace(M, Cc, DEV)
        NC().bn_bwd_dx_red(dy, x, mask, None, None, coef, dx, Cc, 3, x2, mean2, ws2)
        assert torch.equal(dx, dx_ref)
        s1, s2 = _bnr_reference(dres, x2, mean2, torch.ones(M, Cc, dtype=torch.bool))
        got = ws2.double().cpu().sum(0)
        close(got[0], s1, rtol=1e-4, atol=1e-3 * s1.abs().mean().item(), what="sum d")
        close(got[1], s2, rtol=1e-4, atol=1e-3 * s2.abs().mean().item(), what="sum d (x2 - mean2)")


def test_bottleneck_downsample_bn_fused_matches_unfused(monkeypatch):
    """Downsample blocks: bn3's dx sweep writes the shortcut BN's reduce partials and the shortcut BN reads
    dout under bn3's mask (no masked-gradient tensor, no reduce sweep for that BN): two fewer reduce sweeps
    on a two-stage ResNet.  Run in the deterministic mode (fixed-order statistics), so the reference path
    is bitwise reproducible: the forward loss is identical, and the gradients differ only by the shortcut
    BN's reduce summation order (partial rows of the dx sweep vs the reduce sweep's), then bf16 rounding."""
    from noise import rel

    from distributeddeeplearningspark_amd.models.resnet import ResNet
    from distributeddeeplearningspark_amd.ops import fused_blocks as FB
    from distributeddeeplearningspark_amd.ops.determinism import deterministic

    torch.manual_seed(6)
    x = torch.randn(64, 64, 64, 3)
    y = torch.randint(0, 10, (64,))
    out = []
    with deterministic(True):
        for fuse in (False, True, False):
            monkeypatch.setattr(FB, "_FUSE_DOWN", fuse)
            m = ResNet(blocks=(1, 1), input_shape=(64, 64, 3), num_classes=10)
            m.compile("sgd", "sparse_categorical_crossentropy")
            m.place(DEV, seed=7)
            xd, yd = m.to_input(x), m.to_target(y)
            m.backward_step(xd, yd)
            from torch.profiler import ProfilerActivity, profile

            torch.cuda.synchronize()
            with profile(activities=[ProfilerActivity.CUDA]) as prof:
                loss = m.backward_step(xd, yd)
                torch.cuda.synchronize()
            n_reduce = sum(1 for e in prof.events() if "bn_bwd_reduce" in e.name)
            out.append((float(loss.detach()), m.arena.to_canonical(m.arena.grad.detach()).float().cpu().clone(), n_reduce))
    (l0, g0, r0), (l1, g1, r1), (l0b, g0b, _) = out
    assert r1 == r0 - 2, (r1, r0)
    assert l0 == l0b and torch.equal(g0, g0b)  # the reference is reproducible in this mode
    assert l1 == l0, (l1, l0)
    assert rel(g1, g0) < 2e-2, rel(g1, g0)


def test_bottleneck_chain_fused_bn_reduce_matches_unfused(monkeypatch):
    """Two identity-chained bottlenecks at stage-1 shapes (M = 64 x 16 x 16 = 16384 rows: the second
    block's conv1 data-gradient runs on the streaming kernel and accumulates the first block's bn3
    backward sums, whose reduce sweep is then skipped): gradients equal the unfused run's up to that
    run's own spread (tests/noise.py)."""
    from noise import assert_scalar_within_noise, assert_within_noise

    from distributeddeeplearningspark_amd.models.resnet import ResNet
    from distributeddeeplearningspark_amd.ops import fused_blocks as FB

    torch.manual_seed(2)
    x = torch.randn(64, 64, 64, 3)
    y = torch.randint(0, 10, (64,))
    out = []
    for fuse in (False, True, False):
        monkeypatch.setattr(FB, "_FUSE_BNR", fuse)
        m = ResNet(blocks=(2,), input_shape=(64, 64, 3), num_classes=10)
        m.compile("sgd", "sparse_categorical_crossentropy")
        m.place(DEV, seed=3)
        xd, yd = m.to_input(x), m.to_target(y)
        m.backward_step(xd, yd)  # warm-up (workspace pool sizing)
        from torch.profiler import ProfilerActivity, profile

        torch.cuda.synchronize()
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            loss = m.backward_step(xd, yd)
            torch.cuda.synchronize()
        n_reduce = sum(1 for e in prof.events() if "bn_bwd_reduce" in e.name)
        out.append((float(loss.detach()), m.arena.to_canonical(m.arena.grad.detach()).float().cpu().clone(), n_reduce))
    (l0, g0, r0), (l1, g1, r1), (l0b, g0b, _) = out
    assert r1 == r0 - 1, (r1, r0)  # block 1's bn3 reduce sweep was absorbed by block 2's conv1 dgrad
    # the loss is the FORWARD's (both variants run the same forward kernels): its spread is the forward's own
    # BN-statistics noise, amplified by bf16 through the blocks (measured up to 5.6e-3 relative after four
    # blocks, tests/noise.py) — two reference runs under-sample it, hence the 1e-3 relative floor
    assert_scalar_within_noise(l1, l0, l0b, floor=1e-3)
    assert_within_noise(g1, g0, g0b, floor=2e-3, what="arena gradients")


def test_stem_pool_fusion_matches_separate_apply_and_pool(monkeypatch):
    """Stem conv + BN + ReLU + 3x3/2 max pool as one node (the pool applies the BN affine + ReLU on
    load) vs the separate BN-apply sweep + pool: same loss and gradients up to bf16 rounding of the
    applied activation (the fused pool compares fp32 values, the separate path rounded them first)."""
    from distributeddeeplearningspark_amd.models.resnet import ResNet

    torch.manual_seed(3)
    x = torch.randn(8, 64, 64, 3)
    y = torch.randint(0, 10, (8,))
    out = {}
    for fused in ("1", "0"):
        from distributeddeeplearningspark_amd.ops import fused_blocks as FB

        monkeypatch.setattr(FB, "_STEM_POOL", fused == "1")
        m = ResNet(blocks=(1,), input_shape=(64, 64, 3), num_classes=10)
        m.compile("sgd", "sparse_categorical_crossentropy")
        m.place(DEV, seed=4)
        loss = m.backward_step(m.to_input(x), m.to_target(y))
        out[fused] = (float(loss), m.arena.to_canonical(m.arena.grad.detach()).float().cpu().clone(),
                      m.stem.bn._states["moving_mean"].float().cpu().clone())
    (l1, g1, r1), (l0, g0, r0) = out["1"], out["0"]
    assert abs(l1 - l0) < 2e-3 * max(1.0, abs(l0)), (l1, l0)
    assert ((g1 - g0).norm() / g0.norm()).item() < 2e-2
    torch.testing.assert_close(r1, r0)  # the same batch statistics / running-stat update


@pytest.mark.parametrize("N,H,W,K,C", [(16, 56, 56, 128, 256), (8, 14, 14, 512, 1024), (64, 28, 28, 256, 512)])
def test_dgrad_stride2_subgrid_residual(N, H, W, K, C):
    """linear_dgrad with ``rsub=(H, W)``: the residual lives on the stride-2 subgrid and is added only at
    even (i, j) — equal to scattering it to full resolution (zeros elsewhere) and adding that (both the
    streaming kernel, K <= 256, and the LDS-DMA kernel, K = 512)."""
    from distributeddeeplearningspark_amd.ops import gemm as G

    Hs, Ws = (H + 1) // 2, (W + 1) // 2
    M = N * H * W
    dy = rnd(M, K, seed=31)
    w = rnd(K, C, seed=32, scale=K ** -0.5)
    rs = rnd(N * Hs * Ws, C, seed=33)
    out = G.linear_dgrad(dy, w, resid=rs, rsub=(H, W))
    full = torch.zeros(N, H, W, C, dtype=torch.bfloat16, device=DEV)
    full[:, ::2, ::2, :] = rs.view(N, Hs, Ws, C)
    ref = G.linear_dgrad(dy, w, resid=full.view(M, C))
    close(out, ref, rtol=1e-2, atol=1e-2, what="stride-2 residual")
    assert torch.equal(out.view(N, H, W, C)[:, 1::2], ref.view(N, H, W, C)[:, 1::2])


@pytest.mark.parametrize("M,N,K", [(768, 2304, 16384), (256, 64, 200704), (104, 72, 5000)])
def test_splitk_slabs_match_atomics(M, N, K, monkeypatch):
    """fp32 split-K weight gradients through partial slabs + ordered reduce (GemmParams::split_stride)
    equal the fp32-atomic form and the fp32 reference, accumulate into a pre-filled gradient (beta = 1),
    and repeat bit for bit."""
    from distributeddeeplearningspark_amd.ops import gemm as G

    dy = rnd(K, N, seed=51)
    x = rnd(K, M, seed=52)
    g0 = torch.randn(N, M, device=DEV)
    ref = g0 + dy.float().T @ x.float()
    outs = {}
    for slabs in (False, True):
        monkeypatch.setattr(G, "_SPLITK_SLABS", slabs)
        reps = []
        for _ in range(2):
            gw = g0.clone()
            G.linear_wgrad(dy, x, gw)
            reps.append(gw)
        outs[slabs] = reps
    assert torch.equal(outs[True][0], outs[True][1]), "slab split-K must be bitwise reproducible"
    close(outs[True][0], ref, rtol=2e-3, atol=0.5, what="slabs vs fp32")
    close(outs[True][0], outs[False][0], rtol=1e-4, atol=1e-3, what="slabs vs atomics")
