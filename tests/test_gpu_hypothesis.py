"""Hypothesis-generated shapes for the MFMA GEMM (Dense layer path) and the implicit-GEMM
convolution, against the fp32 PyTorch reference on the same bf16-rounded operands.

Shapes are drawn to hit tile edges (M, N, K not multiples of the 128/64/32 tiles, K below
one MFMA step, channel counts that need the 8-wide padding) rather than the ResNet/BERT
shapes the parametrised tests cover.  Examples are capped so the GPU test tier stays fast."""
import pytest
import torch
import torch.nn.functional as F
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

pytestmark = pytest.mark.gpu

SETTINGS = settings(max_examples=25, deadline=None, derandomize=True,
                    suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])


def _close(a, b, what):
    a, b = a.float().cpu(), b.float().cpu()
    rel = ((a - b).norm() / (b.norm() + 1e-12)).item()
    assert rel < 2e-2, f"{what}: rel_l2={rel:.3e}"


@SETTINGS
@given(M=st.integers(1, 700), N=st.integers(1, 300), K=st.integers(1, 400), relu=st.booleans(),
       bias=st.booleans())
def test_linear_any_shape(M, N, K, relu, bias):
    from distributeddeeplearningspark_amd.ops.linear import linear

    g = torch.Generator().manual_seed(M * 7919 + N * 31 + K)
    x = torch.randn(M, K, generator=g).bfloat16().cuda().requires_grad_(True)
    w = (torch.randn(N, K, generator=g) * (K ** -0.5)).bfloat16().cuda()
    b = torch.randn(N, generator=g).cuda() if bias else None
    gw = torch.zeros(N, K, device="cuda")
    gb = torch.zeros(N, device="cuda") if bias else None
    y = linear(x, w, b, relu=relu, grad_w=gw, grad_b=gb)
    dy = torch.randn(M, N, generator=g).bfloat16().cuda()
    y.backward(dy)
    xr = x.detach().float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    br = b.clone().requires_grad_(True) if bias else None
    yr = F.linear(xr, wr, br)
    yr = torch.relu(yr) if relu else yr
    yr.backward(dy.float())
    _close(y, yr, "y")
    _close(x.grad, xr.grad, "dx")
    _close(gw, wr.grad, "dW")
    if bias:
        _close(gb, br.grad, "db")


@SETTINGS
@given(N=st.integers(1, 4), H=st.integers(3, 20), W=st.integers(3, 20), Ci=st.integers(1, 40),
       Co=st.integers(1, 48), k=st.sampled_from([1, 3, 5]), stride=st.sampled_from([1, 2]),
       pad=st.sampled_from([0, 1, 2]))
def test_conv2d_any_shape(N, H, W, Ci, Co, k, stride, pad):
    from distributeddeeplearningspark_amd.ops.conv import conv2d

    if H + 2 * pad < k or W + 2 * pad < k:
        return
    g = torch.Generator().manual_seed(N + 3 * H + 5 * W + 7 * Ci + 11 * Co + 13 * k)
    x = torch.randn(N, H, W, Ci, generator=g).bfloat16().cuda().requires_grad_(True)
    w = (torch.randn(Co, k, k, Ci, generator=g) * (k * k * Ci) ** -0.5).bfloat16().cuda()
    gw = torch.zeros(Co, k, k, Ci, device="cuda")
    y = conv2d(x, w, stride=stride, padding=pad, grad_w=gw)
    dy = torch.randn(y.shape, generator=g).bfloat16().cuda()
    y.backward(dy)
    xr = x.detach().float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=stride, padding=pad)
    yr.backward(dy.float().permute(0, 3, 1, 2))
    _close(y, yr.permute(0, 2, 3, 1), "y")
    _close(x.grad, xr.grad.permute(0, 2, 3, 1), "dx")
    _close(gw, wr.grad.permute(0, 2, 3, 1), "dW")
