"""Persistent GRU / LSTM kernels (csrc/kernels/rnn.hip) vs the fp32 Keras-math reference."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cell", ["gru", "lstm"])
@pytest.mark.parametrize("rs", [False, True])
@pytest.mark.parametrize("B,T,I,H", [(32, 25, 1, 128), (5, 7, 3, 64), (6, 4, 12, 128), (3, 5, 2, 32)])
def test_rnn_native_matches_reference(cell, rs, B, T, I, H):
    from distributeddeeplearningspark_amd.ops import rnn as R
    from distributeddeeplearningspark_amd.ops._native import C

    G = 3 if cell == "gru" else 4
    g = torch.Generator().manual_seed(0)
    x = torch.randn(B, T, I, generator=g)
    W = torch.randn(I, G * H, generator=g) * 0.3
    U = torch.randn(H, G * H, generator=g) * (1.0 / H ** 0.5)
    b = torch.randn(G * H, generator=g) * 0.1
    dy = torch.randn(B, T, H, generator=g) if rs else torch.randn(B, H, generator=g)
    gW, gU, gb = (torch.zeros_like(t, device="cuda") for t in (W, U, b))
    xg = x.cuda().requires_grad_(True)
    y = R.recurrent(cell, xg, W.cuda(), U.cuda(), b.cuda(), grads=(gW, gU, gb), return_sequences=rs)
    y.backward(dy.cuda())
    assert hasattr(C(), "rnn_fwd")
    xr, Wr, Ur, br = (t.clone().requires_grad_(True) for t in (x, W, U, b))
    yr = R.recurrent_ref(cell, xr, Wr, Ur, br, rs)
    yr.backward(dy)
    for a, r, what in [(y, yr, "y"), (xg.grad, xr.grad, "dx"), (gW, Wr.grad, "dW"), (gU, Ur.grad, "dU"),
                       (gb, br.grad, "db")]:
        err = ((a.detach().cpu().float() - r.detach()).norm() / (r.norm() + 1e-12)).item()
        assert err < 1e-4, (what, err)


def test_mse_kernel_matches_reference():
    from distributeddeeplearningspark_amd.ops import loss as L

    g = torch.Generator().manual_seed(1)
    p = torch.randn(37, 3, generator=g)
    t = torch.randn(37, 3, generator=g)
    pg = p.cuda().requires_grad_(True)
    out = L.mean_squared_error(pg, t.cuda())
    (out * 3.0).backward()
    pr = p.clone().requires_grad_(True)
    ref = ((pr - t) ** 2).mean()
    (ref * 3.0).backward()
    assert abs(out.item() - ref.item()) < 1e-5
    assert torch.allclose(pg.grad.cpu(), pr.grad, atol=1e-6)


def test_recurrent_model_trains_in_fp32_on_gpu():
    from distributeddeeplearningspark_amd.models import zoo

    m = zoo.gru_regressor()
    m.compile("adagrad", "mean_squared_error")
    m.place("cuda:0")
    assert m.compute_dtype == torch.float32
    x = torch.rand(32, 25, 1)
    y = torch.rand(32, 1)
    l0 = m.train_on_batch(x, y)
    for _ in range(20):
        l1 = m.train_on_batch(x, y)
    assert l1 < l0
