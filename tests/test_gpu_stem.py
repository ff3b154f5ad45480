"""Space-to-depth ResNet stem (7x7 s2 conv as a 4x4 s1 conv on a block-2 s2d input) vs the
channel-padded implicit-GEMM stem: same forward and the same parameter gradients."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(s2d):
    from distributeddeeplearningspark_amd.models.resnet import ResNet
    from distributeddeeplearningspark_amd.ops import fused_blocks as FB

    old = FB._STEM_S2D
    FB._STEM_S2D = s2d
    try:
        torch.manual_seed(0)
        x = torch.randn(8, 96, 96, 3)
        y = torch.randint(0, 10, (8,))
        m = ResNet(blocks=(1,), input_shape=(96, 96, 3), num_classes=10)
        m.compile("sgd", "sparse_categorical_crossentropy")
        m.place("cuda", seed=1)
        loss = float(m.backward_step(m.to_input(x), m.to_target(y)))
        stem = m.stem.conv.kernel.grad.detach().clone()
        return loss, stem, m.arena.grad.detach().clone()
    finally:
        FB._STEM_S2D = old


def test_stem_s2d_matches_padded_path():
    """The s2d stem accumulates in a different order than the padded one, so its bf16 outputs differ by
    rounding; the gradients are held to the padded path's own run-to-run spread (tests/noise.py) with a
    1 % floor (measured spread of a single two-path comparison: 3.1 % on the stem kernel)."""
    from noise import assert_within_noise

    l0, s0, g0 = _run(False)
    l1, s1, g1 = _run(True)
    l0b, s0b, g0b = _run(False)
    assert abs(l1 - l0) < 1e-2 * max(1.0, abs(l0)), (l1, l0)
    assert_within_noise(s1, s0, s0b, floor=1e-2, what="stem kernel gradient")
    assert_within_noise(g1, g0, g0b, floor=1e-2, what="arena gradients")


def test_s2d_filter_tables_match_torch_relayout():
    """The table-driven HIP gather (forward filter) and scatter-add (gradient) equal the torch pad / permute
    forms bit for bit, on a channel-padded arena view ([64, 7, 7, 8] storage, 3 logical channels)."""
    from distributeddeeplearningspark_amd.ops import fused_blocks as FB
    from distributeddeeplearningspark_amd.ops._native import C

    torch.manual_seed(3)
    store = torch.randn(64, 7, 7, 8, device="cuda").to(torch.bfloat16)
    w = store[..., :3]
    assert not w.is_contiguous()
    assert torch.equal(FB._s2d_weight_dev(w), FB._s2d_weight(w))
    gstore = torch.randn(64, 7, 7, 8, device="cuda")
    gw = gstore[..., :3]
    before = gstore.clone()
    tmp = torch.randn(64, 4, 4, 16, device="cuda")
    tab, ext = FB._s2d_table(gw)
    C().scatter_add_f32(tmp, tab, gw, ext)
    ref = before[..., :3] + FB._s2d_weight_grad(tmp, 3)
    assert torch.equal(gw, ref)
    assert torch.equal(gstore[..., 3:], before[..., 3:])  # the pad channels untouched


def test_zero_ranges_one_launch():
    """zero_ranges zeroes several buffers (16-B vectors + 4-B tails) and nothing around them."""
    from distributeddeeplearningspark_amd.ops._native import C

    big = torch.randn(10_000, device="cuda")
    a, b, c = big[0:1001], big[1004:3004], big[3008:3013]  # 1001 / 2000 / 5 floats, 16-B aligned starts
    keep = big.clone()
    C().zero_ranges([a, b, c, torch.empty(0, device="cuda")])
    zero = torch.zeros_like(big, dtype=torch.bool)
    zero[0:1001] = zero[1004:3004] = zero[3008:3013] = True
    assert (big[zero] == 0).all()
    assert torch.equal(big[~zero], keep[~zero])
