"""Weight-stationary streaming GEMM (csrc/kernels/gemm_stream.hip) vs an fp32 PyTorch reference:
every (panel width, K) instantiation, K- and row-contiguous weights, ragged M, and the fused
epilogues the ResNet path uses (bias / residual / ReLU / BN statistics)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(M, N, K, b_mode, *, bias=False, resid=False, relu=False, stats=False, alpha=1.0):
    from distributeddeeplearningspark_amd.ops import gemm as G
    from distributeddeeplearningspark_amd.ops._native import C

    g = torch.Generator(device="cuda").manual_seed(M + 7 * N + 13 * K)
    A = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    W = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(torch.bfloat16)
    Wop = W if b_mode == G.KC else W.t().contiguous()
    ldb = K if b_mode == G.KC else N
    b = torch.randn(N, device="cuda", generator=g) if bias else None
    r = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16) if resid else None
    st = torch.zeros(32, 2, N, device="cuda") if stats else None
    out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    G.gemm(A, Wop, out, M, N, K, G.KC, b_mode, K, ldb, N, G.EPI_BF16, alpha=alpha, bias=b, resid=r, ldr=N if resid else 0,
           relu=relu, stats=st, tile=G.TILE_STREAM)
    ref = alpha * (A.float() @ W.float().t())
    if bias:
        ref = ref + b
    if resid:
        ref = ref + r.float()
    if relu:
        ref = ref.clamp_min(0)
    err = ((out.float() - ref).norm() / ref.norm()).item()
    assert err < 8e-3, (M, N, K, b_mode, err)
    if stats:
        o = out.float()
        s = st.sum(0)
        torch.testing.assert_close(s[0], o.sum(0), rtol=1e-3, atol=1e-2 * M ** 0.5)
        torch.testing.assert_close(s[1], (o * o).sum(0), rtol=1e-3, atol=1e-2 * M ** 0.5)
    torch.cuda.synchronize()
    _ = C
    return out


@pytest.mark.parametrize("N,K", [(64, 64), (256, 64), (128, 64), (64, 128), (256, 128), (512, 128), (128, 256),
                                 (64, 256), (1024, 64)])
@pytest.mark.parametrize("b_mode", [0, 1])
def test_stream_shapes(N, K, b_mode):
    _run(20000 + 37, N, K, b_mode)


@pytest.mark.parametrize("N,K", [(256, 64), (512, 128), (128, 256), (64, 64)])
def test_stream_epilogues(N, K):
    _run(33333, N, K, 0, bias=True, relu=True, stats=True, alpha=0.5)
    _run(33333, N, K, 1, resid=True, stats=True)
    _run(4096 + 5, N, K, 0, resid=True, relu=True)


def test_stream_auto_selected_and_matches_tile_kernel():
    from distributeddeeplearningspark_amd.ops import gemm as G

    M, N, K = 50000, 256, 64
    assert G.use_stream(M, N, K, G.KC, G.KC, G.EPI_BF16, K, N)
    A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    W = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    o1 = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    o2 = torch.empty_like(o1)
    G.gemm(A, W, o1, M, N, K, G.KC, G.KC, K, K, N, G.EPI_BF16, tile=G.TILE_STREAM)
    G.gemm(A, W, o2, M, N, K, G.KC, G.KC, K, K, N, G.EPI_BF16, tile=0)
    assert torch.equal(o1, o2)  # same fp32 accumulation order per element -> identical bf16
