"""BN-backward reduction fused into the data-gradient GEMM epilogue (ACT_BN_BWD): the stored
gradient is ReLU-masked by the BN input and the shard rows hold (sum d', sum d'(x - mean)).
Covered on both GEMM families that produce ResNet data-gradients: the 128-tile kernel and the
weight-stationary streaming kernel (skinny K, M >= 16384)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,N,K", [(3000, 64, 512), (20000, 64, 256), (20000, 128, 128), (700, 256, 1024)])
def test_linear_dgrad_bn_bwd_epilogue(M, N, K):
    from distributeddeeplearningspark_amd.ops import gemm as G

    g = torch.Generator().manual_seed(M + N + K)
    dy = torch.randn(M, K, generator=g).bfloat16().cuda()       # gradient of the next layer's output
    w = (torch.randn(K, N, generator=g) * K ** -0.5).bfloat16().cuda()
    x = torch.randn(M, N, generator=g).bfloat16().cuda()         # BN input (conv output)
    ssm = torch.stack([torch.rand(N, generator=g) + 0.5, torch.randn(N, generator=g) * 0.3,
                       torch.randn(N, generator=g) * 0.1]).cuda()
    stats = torch.zeros(32, 2, N, device="cuda")
    out = G.linear_dgrad(dy, w, bn_bwd=(x, ssm), stats=stats)
    d = (dy.float() @ w.float()).bfloat16().float()
    xf = x.float()
    keep = (xf * ssm[0] + ssm[1]) > 0
    ref = torch.where(keep, d, torch.zeros_like(d))
    err = ((out.float() - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err
    o = out.float()
    s1, s2 = stats.sum(0)
    r1, r2 = o.sum(0), (o * (xf - ssm[2])).sum(0)
    assert torch.allclose(s1, r1, rtol=1e-3, atol=1e-2 * r1.abs().max().item()), (s1 - r1).abs().max()
    assert torch.allclose(s2, r2, rtol=1e-3, atol=1e-2 * r2.abs().max().item()), (s2 - r2).abs().max()


def test_bottleneck_backward_with_epilogue_matches_unfused(monkeypatch):
    """Whole fused bottleneck: parameter gradients with the epilogue reduction equal the ones
    computed with the separate BN-backward sweeps (DDL_BN_BWD_EPILOGUE=0)."""
    from distributeddeeplearningspark_amd.models.resnet import Bottleneck
    from distributeddeeplearningspark_amd.ops import conv as CV
    from distributeddeeplearningspark_amd.ops.norm import reset_workspaces

    res = []
    for fuse in (True, False):
        monkeypatch.setattr(CV, "_BN_EPI", fuse)  # opt-in path vs the default sweeps
        torch.manual_seed(0)
        from distributeddeeplearningspark_amd.models.core import Sequential  # noqa: F401

        blk = Bottleneck(64, strides=1, downsample=True, name="blk")
        blk.ensure_built((28, 28, 128))
        from distributeddeeplearningspark_amd.models.params import ParamArena

        arena = ParamArena(blk.all_params(), torch.device("cuda"), torch.bfloat16, seed=3)
        blk.states_to("cuda")
        x = (torch.randn(8, 28, 28, 128, generator=torch.Generator().manual_seed(1))).bfloat16().cuda()
        x.requires_grad_(True)
        reset_workspaces("cuda")
        arena.zero_grad()
        y = blk.call(x, training=True)
        y.backward(torch.randn(y.shape, generator=torch.Generator().manual_seed(2)).bfloat16().cuda())
        torch.cuda.synchronize()
        res.append((arena.grad.detach().clone(), x.grad.detach().float().clone()))
    (g1, dx1), (g0, dx0) = res
    assert ((g1 - g0).norm() / g0.norm()).item() < 2e-2
    assert ((dx1 - dx0).norm() / dx0.norm()).item() < 2e-2
