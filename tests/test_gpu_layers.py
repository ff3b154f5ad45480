"""GPU numerics of the Keras layer kernels (csrc/kernels/layer_ops.hip, gemm_f32.hip, the generic
recurrent cells of rnn.hip) against plain PyTorch fp32 references of the same op, and a check
that a GPU model built from these layers launches only the framework's HIP kernels."""
import pytest
import numpy as np
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _C():
    from distributeddeeplearningspark_amd.ops._native import C

    return C()


# ------------------------------------------------------------------------------- fp32 GEMM
@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (800, 384, 25), (77, 130, 513), (128, 64, 16), (5, 300, 1)])
@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True), (True, True)])
def test_gemm_f32_strides(M, N, K, ta, tb):
    g = torch.Generator(device=DEV).manual_seed(M * 7 + N)
    A = torch.randn(M, K, device=DEV, generator=g)
    B = torch.randn(K, N, device=DEV, generator=g)
    a = A.t().contiguous() if ta else A  # stored transposed: A(m,k) = a[k*M + m]
    b = B.t().contiguous() if tb else B
    sam, sak = (1, M) if ta else (K, 1)
    sbk, sbn = (1, K) if tb else (N, 1)
    bias = torch.randn(N, device=DEV, generator=g)
    C0 = torch.randn(M, N, device=DEV, generator=g)
    c = C0.clone()
    _C().gemm_f32(a, sam, sak, b, sbk, sbn, c, N, M, N, K, 0.5, 1.0, bias, True)
    ref = torch.relu(0.5 * (A.double() @ B.double()) + C0.double() + bias.double())
    torch.testing.assert_close(c.double(), ref, rtol=1e-5, atol=1e-4)


# ------------------------------------------------------------------------------- activations
ACTS = ["relu", "tanh", "sigmoid", "hard_sigmoid", "elu", "selu", "softplus", "gelu"]


@pytest.mark.parametrize("name", ACTS + ["softmax"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_activation_kernels(name, dtype):
    from distributeddeeplearningspark_amd.ops import act as A

    g = torch.Generator(device=DEV).manual_seed(3)
    x0 = (torch.randn(37, 70, device=DEV, generator=g) * 3).to(dtype)
    dy = torch.randn(37, 70, device=DEV, generator=g).to(dtype)
    x = x0.clone().requires_grad_(True)
    y = A.activation(x, name)
    y.backward(dy)
    xr = x0.float().clone().requires_grad_(True)
    yr = A.activation_ref(name, xr)
    yr.backward(dy.float())
    tol = dict(rtol=2e-2, atol=2e-2) if dtype == torch.bfloat16 else dict(rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(y.float(), yr, **tol)
    gx, gr = x.grad.float(), xr.grad
    if name == "hard_sigmoid":  # derivative from the (rounded) output: compare away from the clip kinks
        keep = (x0.float().abs() - 2.5).abs() > 0.1
        gx, gr = gx[keep], gr[keep]
    torch.testing.assert_close(gx, gr, **tol)


def test_dropout_kernel_mask_and_backward():
    from distributeddeeplearningspark_amd.ops import act as A

    x = torch.ones(1 << 20, device=DEV).requires_grad_(True)
    y = A.dropout(x, 0.25, True, seed=1234)
    kept = (y != 0).float()
    frac = float(kept.mean())
    assert abs(frac - 0.75) < 0.005, frac
    torch.testing.assert_close(y[y != 0], torch.full_like(y[y != 0], 1 / 0.75))
    y.backward(torch.ones_like(y))
    torch.testing.assert_close(x.grad, kept / 0.75)  # same mask regenerated in backward
    y2 = A.dropout(x.detach(), 0.25, True, seed=1234)
    assert torch.equal(y2, y.detach())
    assert A.dropout(x, 0.25, False) is x


@pytest.mark.parametrize("k,s,p", [((2, 2), (2, 2), (0, 0)), ((3, 3), (1, 1), (1, 1)), ((3, 3), (2, 2), (1, 1)),
                                   ((2, 3), (1, 2), (0, 1))])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_avgpool2d_kernel(k, s, p, dtype):
    from distributeddeeplearningspark_amd.ops import act as A

    g = torch.Generator(device=DEV).manual_seed(5)
    x0 = torch.randn(3, 11, 9, 20, device=DEV, generator=g).to(dtype)
    x = x0.clone().requires_grad_(True)
    y = A.avg_pool2d(x, k, s, p)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x0.double().cpu().requires_grad_(True)  # CPU fp64 reference
    yr = A.avgpool_ref(xr, k, s, p)
    yr.backward(dy.double().cpu())
    tol = dict(rtol=2e-2, atol=2e-2) if dtype == torch.bfloat16 else dict(rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(y.double().cpu(), yr.detach(), **tol)
    torch.testing.assert_close(x.grad.double().cpu(), xr.grad, **tol)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_embedding_kernel(dtype):
    from distributeddeeplearningspark_amd.ops.embedding import embedding

    g = torch.Generator(device=DEV).manual_seed(9)
    W = torch.randn(50, 24, device=DEV, generator=g).to(dtype)
    ids = torch.randint(0, 50, (6, 13), device=DEV, generator=g)
    gw = torch.zeros(50, 24, device=DEV)
    w = W.clone().requires_grad_(True)  # as in the arena: compute weights anchor the autograd graph
    out = embedding(ids, w, grad_w=gw)
    torch.testing.assert_close(out.float(), W.float()[ids])
    dy = torch.randn_like(out)
    out.backward(dy)
    ref = torch.zeros(50, 24, device=DEV).index_add_(0, ids.reshape(-1), dy.float().reshape(-1, 24))
    torch.testing.assert_close(gw, ref, rtol=1e-5, atol=1e-5)


# ------------------------------------------------------------------------------- recurrent cells
@pytest.mark.parametrize("cell,H,act,ract", [("rnn", 32, "tanh", "hard_sigmoid"), ("rnn", 100, "relu", "sigmoid"),
                                             ("gru", 32, "tanh", "sigmoid"), ("lstm", 96, "tanh", "sigmoid"),
                                             ("gru", 128, "relu", "hard_sigmoid"), ("lstm", 48, "elu", "hard_sigmoid"),
                                             ("gru", 24, "tanh", "hard_sigmoid")])
@pytest.mark.parametrize("rs", [False, True])
def test_generic_recurrent_kernels(cell, H, act, ract, rs):
    from distributeddeeplearningspark_amd.ops import rnn as R

    G = {"rnn": 1, "gru": 3, "lstm": 4}[cell]
    B, T, I = 5, 7, 3
    g = torch.Generator(device=DEV).manual_seed(H + G)
    x0 = torch.randn(B, T, I, device=DEV, generator=g)
    W = torch.randn(I, G * H, device=DEV, generator=g) * 0.3
    U = torch.randn(H, G * H, device=DEV, generator=g) * (0.5 / H ** 0.5)
    b = torch.randn(G * H, device=DEV, generator=g) * 0.1
    gW, gU, gb = torch.zeros_like(W), torch.zeros_like(U), torch.zeros_like(b)
    x = x0.clone().requires_grad_(True)
    y = R.recurrent(cell, x, W, U, b, grads=(gW, gU, gb), return_sequences=rs, activation=act,
                    recurrent_activation=ract)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr, Wr, Ur, br = (t.detach().double().requires_grad_(True) for t in (x0, W, U, b))
    yr = R.recurrent_ref(cell, xr, Wr, Ur, br, rs, act, ract)
    yr.backward(dy.double())
    torch.testing.assert_close(y.double(), yr, rtol=1e-4, atol=1e-5)
    for got, ref in ((x.grad, xr.grad), (gW, Wr.grad), (gU, Ur.grad), (gb, br.grad)):
        torch.testing.assert_close(got.double(), ref, rtol=1e-3, atol=1e-4)


# ------------------------------------------------------------------------------- fp32 Dense
def test_fp32_dense_on_gemm_f32():
    from distributeddeeplearningspark_amd.ops.linear import linear

    g = torch.Generator(device=DEV).manual_seed(11)
    x0 = torch.randn(33, 17, device=DEV, generator=g)
    w = torch.randn(9, 17, device=DEV, generator=g)
    b = torch.randn(9, device=DEV, generator=g)
    gw, gb = torch.zeros_like(w), torch.zeros_like(b)
    x = x0.clone().requires_grad_(True)
    y = linear(x, w, b, relu=True, grad_w=gw, grad_b=gb)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr, wr, br = (t.clone().double().requires_grad_(True) for t in (x0, w, b))
    yr = torch.relu(xr @ wr.t() + br)
    yr.backward(dy.double())
    torch.testing.assert_close(y.double(), yr, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(x.grad.double(), xr.grad, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(gw.double(), wr.grad, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(gb.double(), br.grad, rtol=1e-5, atol=1e-5)


# ------------------------------------------------------------------------------- no torch kernels
def _kernel_names(fn):
    from torch.profiler import ProfilerActivity, profile

    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        fn()
        torch.cuda.synchronize()
    return {e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA}


# torch kernels that would mean a layer's COMPUTE fell back to ATen / MIOpen / hipBLASLt.  Glue
# that stays in ATen (copies into static buffers, memsets, the scalar loss mean) is not listed.
_DENY = ("tanh", "sigmoid", "elu", "gelu", "softplus", "softmax", "dropout", "bernoulli", "avg_pool", "AvgPool",
         "avgpool", "embedding", "index_add", "indexing_backward", "Cijk", "gemm", "Gemm", "addmm", "nll", "max_pool",
         "MaxPool", "miopen", "rnn", "lstm", "gru", "relu", "threshold", "erf", "exp_kernel", "sort", "rocprim",
         "radix", "layer_norm", "LayerNorm", "cross_entropy", "log_softmax")


@pytest.mark.parametrize("which", ["dense_dropout", "embed_rnn", "avgpool_cnn"])
def test_layer_models_run_only_hip_kernels(which):
    from distributeddeeplearningspark_amd.models import layers as L
    from distributeddeeplearningspark_amd.models.core import Sequential

    torch.manual_seed(0)
    if which == "dense_dropout":
        m = Sequential([L.Dense(64, input_shape=(20,), activation="tanh"), L.Dropout(0.3), L.Activation("sigmoid"),
                        L.Dense(32, activation="elu"), L.Dense(10), L.Activation("softmax")])
        x, y = torch.randn(16, 20), torch.randint(0, 10, (16,))
        loss = "sparse_categorical_crossentropy"
    elif which == "embed_rnn":
        m = Sequential([L.Embedding(100, 16, input_shape=(12,)), L.SimpleRNN(32, activation="relu"),
                        L.Dense(1, activation="sigmoid")])
        x, y = torch.randint(0, 100, (8, 12)), torch.rand(8, 1)
        loss = "mean_squared_error"
    else:
        m = Sequential([L.Conv2D(16, (3, 3), input_shape=(12, 12, 8), padding="same"), L.Activation("relu"),
                        L.AveragePooling2D((2, 2)), L.Flatten(), L.Dense(10, activation="softmax")])
        x, y = torch.randn(4, 12, 12, 8), torch.randint(0, 10, (4,))
        loss = "sparse_categorical_crossentropy"
    m.compile("adam", loss)
    m.place(DEV, seed=0)
    xd, yd = m.to_input(x), m.to_target(y)
    m.train_on_batch(xd, yd)  # warm-up (lazy workspaces)
    names = _kernel_names(lambda: m.train_on_batch(xd, yd))
    fallen = sorted(n for n in names if "ddl::" not in n and any(d in n for d in _DENY))
    assert not fallen, f"layer compute ran on torch kernels: {fallen}"
    assert any("ddl::" in n for n in names)


def _bert_tiny():
    from distributeddeeplearningspark_amd.models.bert import BertConfig, BertForMaskedLM

    m = BertForMaskedLM(BertConfig.tiny(vocab_size=1100, max_position_embeddings=128))
    m.compile("adamw", "sparse_categorical_crossentropy")
    m.place(DEV, seed=0)
    return m


@pytest.mark.parametrize("with_count", [True, False])
def test_bert_tiny_train_step_runs_only_hip_kernels(with_count):
    """BERT-tiny MLM step (embeddings, encoder, head, xent, AdamW): no GEMM library, no erf/exp GELU
    backward, no id sort, no LayerNorm / cross-entropy fallback.  ``with_count=False`` drops
    ``num_masked`` so the loss normaliser is counted on the device (no host sync either)."""
    from distributeddeeplearningspark_amd.data.synthetic import mlm_batch

    m = _bert_tiny()
    x, y = mlm_batch(4, 128, 1100, max_predictions=8, seed=1)
    if not with_count:
        y = {k: v for k, v in y.items() if k != "num_masked"}
    xd, yd = m.to_input(x), m.to_target(y)
    l0 = float(m.train_on_batch(xd, yd))
    names = _kernel_names(lambda: m.train_on_batch(xd, yd))
    fallen = sorted(n for n in names if "ddl::" not in n and any(d in n for d in _DENY))
    assert not fallen, f"BERT compute ran on library kernels: {fallen}"
    assert any("embed_word_grad_atomic" in n for n in names)
    assert l0 == l0 and abs(l0 - np.log(1100)) < 1.5


def test_bert_tiny_predict_runs_only_hip_kernels():
    """Full-sequence MLM inference (the partition predictor's path): the head runs on the HIP GEMM
    epilogues + LayerNorm, and matches the fp32 CPU reference head on the same encoder output."""
    from distributeddeeplearningspark_amd.data.synthetic import mlm_batch
    from distributeddeeplearningspark_amd.models.bert import mlm_head_ref

    m = _bert_tiny()
    x, _ = mlm_batch(2, 128, 1100, max_predictions=8, seed=2)
    xd = m.to_input(x)
    lg = m.forward(xd)
    names = _kernel_names(lambda: m.forward(xd))
    fallen = sorted(n for n in names if "ddl::" not in n and any(d in n for d in _DENY))
    assert not fallen, f"BERT predict ran on library kernels: {fallen}"
    assert lg.shape == (2, 128, 1100) and lg.dtype == torch.float32
    with torch.no_grad():
        h = m.encode(xd, False).float().cpu()
        hd = m.head
        ref = mlm_head_ref(h, hd.t_w.master.cpu(), hd.t_b.master.cpu(), hd.ln_g.master.cpu(), hd.ln_b.master.cpu(),
                           m.embeddings.word.master.cpu(), hd.dec_b.master.cpu(), m.config.layer_norm_eps, 1100)
    err = (lg.reshape(-1, 1100).cpu() - ref).abs().max().item()
    assert err < 0.05 * ref.abs().max().item() + 0.05, err


def test_sequential_fused_convbn_matches_two_node_path(monkeypatch):
    """Sequential Conv2D -> BatchNormalization -> ReLU trains through ONE fused autograd node
    (ops/fused_blocks.py, models/core.py:_convbn_unit) — VGG-style blocks incl. a 3-channel input, a
    stride-2 "same" conv (asymmetric padding: keeps the two-node path) and a 2x2 pool: same loss,
    gradients and BN running statistics as the two-node path (DDL_FUSE_CONVBN=0)."""
    from distributeddeeplearningspark_amd.models import layers as L
    from distributeddeeplearningspark_amd.models.core import Sequential

    def build():
        torch.manual_seed(0)
        m = Sequential([L.Conv2D(64, (3, 3), input_shape=(16, 16, 3), padding="same", use_bias=False),
                        L.BatchNormalization(momentum=0.9, epsilon=1e-5), L.Activation("relu"),
                        L.Conv2D(64, (3, 3), padding="same", use_bias=False), L.BatchNormalization(), L.Activation("relu"),
                        L.MaxPooling2D((2, 2)),
                        L.Conv2D(128, (3, 3), strides=2, padding="same", use_bias=False), L.BatchNormalization(),
                        L.Activation("relu"),
                        L.Conv2D(128, (3, 3), padding="same", use_bias=False), L.BatchNormalization(),
                        L.Flatten(), L.Dense(10, activation="softmax")])
        m.compile("sgd", "sparse_categorical_crossentropy")
        m.place(DEV, seed=0)
        return m

    g = torch.Generator().manual_seed(1)
    x, y = torch.randn(8, 16, 16, 3, generator=g), torch.randint(0, 10, (8,), generator=g)
    res = {}
    for fuse in ("1", "0"):
        from distributeddeeplearningspark_amd.models import core as _core

        monkeypatch.setattr(_core, "FUSE_CONVBN", fuse == "1")
        m = build()
        xd, yd = m.to_input(x), m.to_target(y)
        loss = float(m.backward_step(xd, yd))
        stats = [l._states["moving_mean"].float().cpu().clone() for l in m.layers if isinstance(l, L.BatchNormalization)]
        res[fuse] = (loss, m.arena.to_canonical(m.arena.grad.detach()).float().cpu().clone(), stats)
        if fuse == "1":
            assert len(m.__dict__.get("_convbn_units", {})) == 3  # the stride-2 conv keeps two nodes
    (l1, g1, s1), (l0, g0, s0) = res["1"], res["0"]
    assert abs(l1 - l0) < 1e-3 * abs(l0), (l1, l0)
    rel = ((g1 - g0).norm() / g0.norm()).item()
    assert rel < 1e-2, rel
    for a, b in zip(s1, s0):
        assert torch.allclose(a, b, rtol=1e-3, atol=1e-4)


def test_sequential_conv_chain_fuses_bn_backward_reduce(monkeypatch):
    """VGG block conv -> BN -> ReLU -> conv -> BN -> ReLU -> conv -> BN -> ReLU -> 2x2 pool: each conv's
    data-gradient epilogue accumulates the previous BN's backward partial sums (mode 2: ReLU recomputed
    from its input) and the last BN's reduce and dx sweeps run through the pool's argmax
    (``_ConvBNPoolFn``), so no BN runs a separate reduce sweep (3 without the fusions); loss and
    gradients as without them (fp32 summation order only)."""
    from distributeddeeplearningspark_amd.models import layers as L
    from distributeddeeplearningspark_amd.models.core import Sequential
    from distributeddeeplearningspark_amd.ops import fused_blocks as FB
    from distributeddeeplearningspark_amd.ops._native import C

    def build():
        torch.manual_seed(0)
        m = Sequential([L.Conv2D(64, (3, 3), input_shape=(32, 32, 8), padding="same", use_bias=False),
                        L.BatchNormalization(), L.Activation("relu"),
                        L.Conv2D(128, (3, 3), padding="same", use_bias=False), L.BatchNormalization(), L.Activation("relu"),
                        L.Conv2D(128, (3, 3), padding="same", use_bias=False), L.BatchNormalization(), L.Activation("relu"),
                        L.MaxPooling2D((2, 2)), L.Flatten(), L.Dense(10, activation="softmax")])
        m.compile("sgd", "sparse_categorical_crossentropy")
        m.place(DEV, seed=0)
        return m

    calls = []
    native = C()
    orig = native.bn_bwd_reduce
    monkeypatch.setattr(native, "bn_bwd_reduce", lambda *a, **k: (calls.append(1), orig(*a, **k))[1])
    g = torch.Generator().manual_seed(2)
    x, y = torch.randn(64, 32, 32, 8, generator=g), torch.randint(0, 10, (64,), generator=g)
    from noise import assert_within_noise

    res = {}
    for run, fuse in (("fused", True), ("plain", False), ("plain2", False)):
        monkeypatch.setattr(FB, "_FUSE_BNR", fuse)
        monkeypatch.setattr(FB, "_SEQ_POOL", fuse)
        calls.clear()
        m = build()
        loss = float(m.backward_step(m.to_input(x), m.to_target(y)).detach())
        res[run] = (loss, m.arena.to_canonical(m.arena.grad.detach()).float().cpu().clone(), len(calls))
    (l1, g1, n1), (l0, g0, n0), (_, g0b, _) = res["fused"], res["plain"], res["plain2"]
    assert (n1, n0) == (0, 3), (n1, n0)
    assert abs(l1 - l0) < 1e-4 * abs(l0), (l1, l0)
    # the fused sums are taken before the bf16 rounding of the data-gradient (the sweep sums the rounded
    # tensor): measured 4.4e-3 relative on these gradients, against the plain path's own atomics spread
    assert_within_noise(g1, g0, g0b, floor=2e-3, what="parameter gradients")


def test_mnist_cnn_padded_arena_matches_fp32_cpu():
    """The reference's MNIST CNN (``ddl_mnist_aztk.py:180-192``: 1-channel input, Dense(225), Dense(10))
    on the GPU keeps its odd-width weights in zero-padded arena storage (params.py) and passes padded
    activations / gradients between layers (ops/zpad.py): same loss and parameter gradients as the fp32 CPU
    model, padding that stays exactly zero through an Adam step, and a training step that launches no
    ATen kernel besides the eager step's gradient zero-fill and the loss read-back."""
    from distributeddeeplearningspark_amd.models.zoo import mnist_cnn

    def build(dev):
        m = mnist_cnn()
        m.compile("adam", "categorical_crossentropy")
        m.place(dev, seed=0)
        return m

    mg, mc = build(DEV), build("cpu")
    padded = [p for p in mg.arena.params if p.padded]
    assert len(padded) == 5, padded  # conv1 kernel (1 -> 8 channels), both Dense kernels and biases
    g = torch.Generator().manual_seed(3)
    x = torch.rand(16, 28, 28, 1, generator=g)
    y = F.one_hot(torch.randint(0, 10, (16,), generator=g), 10).float()
    lg = float(mg.backward_step(mg.to_input(x), mg.to_target(y)))
    lc = float(mc.backward_step(mc.to_input(x), mc.to_target(y)))
    assert abs(lg - lc) < 0.02 * abs(lc) + 1e-3, (lg, lc)
    errs = {}
    for pg, pc in zip(mg.arena.params, mc.arena.params):
        a, b = pg.grad.float().cpu(), pc.grad.float()
        errs[pg.name] = (a - b).norm().item() / max(b.norm().item(), 1e-6)
    print("relative gradient error vs fp32 CPU:", {k: round(v, 4) for k, v in errs.items()})
    # bf16 activations / gradients: the first conv's weight gradient sits under the longest bf16 chain (~7 %);
    # a layout error (a tap or channel misread) would be O(1)
    assert max(errs.values()) < 0.1, errs

    def pad_max(p, t):
        m = torch.ones(p.pshape, dtype=torch.bool)
        m[p.logical] = False
        return t.detach().float().cpu()[m].abs().max().item()

    for p in padded:
        assert pad_max(p, p.pgrad) == 0.0 and pad_max(p, p.pmaster) == 0.0, p.name
    mg.optimizer.step(1.0)
    for p in padded:
        assert pad_max(p, p.pmaster) == 0.0 and pad_max(p, p.pdata) == 0.0, p.name
    xd, yd = mg.to_input(x), mg.to_target(y)
    mg.train_on_batch(xd, yd)
    names = _kernel_names(lambda: mg.train_on_batch(xd, yd))
    aten = sorted(n for n in names if "ddl::" not in n and "Memcpy" not in n and "FillFunctor<float>" not in n)
    assert not aten, f"ATen kernels in the MNIST step: {aten}"


def test_derived_filters_one_launch_matches_per_copy():
    """ops/derived.py: the step's flipped / class / transposed weight copies come from ONE taps_batch launch
    (from the second step on) and give bit-identical gradients to the one-launch-per-copy path (deterministic
    mode), for a ResNet stage with stride-2 and 3x3 convs and a Dense head over 4096+ rows."""
    from distributeddeeplearningspark_amd.models.resnet import ResNet
    from distributeddeeplearningspark_amd.ops import derived
    from distributeddeeplearningspark_amd.ops import determinism as D

    torch.manual_seed(0)
    x = torch.randn(8, 32, 32, 3)
    y = torch.randint(0, 10, (8,))
    grads = {}
    D.set_enabled(True)
    try:
        for on in (True, False):
            derived.ENABLED = on
            m = ResNet(blocks=(1, 1), input_shape=(32, 32, 3), num_classes=10)
            m.compile("sgd", "sparse_categorical_crossentropy")
            m.place(DEV, seed=5)
            xd, yd = m.to_input(x), m.to_target(y)
            m.train_on_batch(xd, yd)  # step 1 registers the copies, one launch each
            names = _kernel_names(lambda: m.backward_step(xd, yd))
            grads[on] = m.arena.grad.detach().float().cpu().clone()
            if on:
                assert any("taps_batch_kernel" in n for n in names), sorted(names)
                assert not any("filter_taps_transpose" in n or "transpose_bf16" in n for n in names), sorted(names)
    finally:
        derived.ENABLED = True
        D.set_enabled(False)
    assert torch.equal(grads[True], grads[False])


def test_taps_batch_mixed_jobs_match_reference():
    """csrc/kernels/layer_ops.hip taps_batch: one launch over a job table mixing 64-multiple plain transposes
    (the 16-B vector path: BERT-base weight shapes), odd-sized transposes and tap-reordered conv filters."""
    c = _C()
    g = torch.Generator(device=DEV).manual_seed(7)
    srcs, dsts, taps, refs = [], [], [], []
    for R, Cc in ((768, 3072), (2304, 768), (1000, 2048), (40, 24)):
        w = torch.randn(R, Cc, device=DEV, generator=g).to(torch.bfloat16)
        srcs.append(w)
        dsts.append(torch.empty(Cc, R, dtype=torch.bfloat16, device=DEV))
        taps.append([0])
        refs.append(w.t())
    for Co, Ci, tp in ((64, 32, list(range(8, -1, -1))), (24, 16, [0, 2, 6, 8]), (128, 64, list(range(8, -1, -1))),
                       (64, 128, [4, 3, 5, 1, 7, 0, 2, 6, 8]), (128, 128, [4, 1, 7])):
        w = torch.randn(Co, 3, 3, Ci, device=DEV, generator=g).to(torch.bfloat16)
        srcs.append(w)
        dsts.append(torch.empty(Ci, len(tp), Co, dtype=torch.bfloat16, device=DEV))
        taps.append(tp)
        refs.append(w.reshape(Co, 9, Ci)[:, tp, :].permute(2, 1, 0))
    table, blocks = c.taps_batch_table(srcs, dsts, taps)
    c.taps_batch(table.to(DEV), len(srcs), int(blocks))
    for d, r in zip(dsts, refs):
        assert torch.equal(d, r.reshape(d.shape)), d.shape
