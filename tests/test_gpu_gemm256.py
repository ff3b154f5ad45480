"""The 256x256 ping-pong GEMM kernel (csrc/include/ddl_gemm256.h) against fp32 references: every operand
layout, every epilogue, tails in M and N, split-K (atomics and partial slabs)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


TILES = [4]  # G.TILE256


def rnd(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16).to(DEV)


def close(a, b, rtol=2e-2, atol=2e-2, what=""):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs()
    bad = (err > atol + rtol * b.abs()).float().mean().item()
    rel = (err.norm() / (b.norm() + 1e-12)).item()
    assert bad < 1e-3 and rel < 2e-2, f"{what}: frac_bad={bad:.2e} rel={rel:.2e}"


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 768), (1000, 520, 256), (300, 2304, 128),
                                   (4096, 256, 1024), (4200, 4104, 192)])
@pytest.mark.parametrize("a_rc", [False, True])
@pytest.mark.parametrize("b_rc", [False, True])
@pytest.mark.parametrize("tile", TILES)
def test_gemm256_layouts(M, N, K, a_rc, b_rc, tile):
    from distributeddeeplearningspark_amd.ops import gemm as G

    if (a_rc and M % 8) or (b_rc and N % 8):
        pytest.skip("row-contiguous operands need a multiple of 8 rows")
    A, B = rnd(M, K, seed=1), rnd(N, K, seed=2)
    ref = A.float() @ B.float().T
    a_t = A.T.contiguous() if a_rc else A
    b_t = B.T.contiguous() if b_rc else B
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    G.gemm(a_t, b_t, out, M, N, K, G.RC if a_rc else G.KC, G.RC if b_rc else G.KC, a_t.stride(0), b_t.stride(0), N,
           G.EPI_BF16, tile=tile)
    close(out, ref, what=f"tile {tile} {M}x{N}x{K} a_rc={a_rc} b_rc={b_rc}")


@pytest.mark.parametrize("tile", TILES)
def test_gemm256_epilogues(tile):
    from distributeddeeplearningspark_amd.ops import gemm as G
    from distributeddeeplearningspark_amd.ops import transformer as T

    M, N, K = (4352, 4096, 256) if tile == 9 else (768, 1024, 512)  # persistent: 272 tiles
    A, B = rnd(M, K, seed=3), rnd(N, K, seed=4, scale=0.1)
    bias = torch.randn(N, device=DEV) * 0.1
    res = rnd(M, N, seed=5)
    pre_r = A.float() @ B.float().T + bias
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    G.gemm(A, B, out, M, N, K, G.KC, G.KC, K, K, N, G.EPI_BF16, bias=bias, resid=res, ldr=N, relu=True,
           tile=tile)
    close(out, torch.relu(pre_r + res.float()), what="bias+resid+relu")
    aux = torch.empty_like(out)
    G.gemm(A, B, out, M, N, K, G.KC, G.KC, K, K, N, G.EPI_BF16, bias=bias, relu=G.ACT_GELU, aux=aux, tile=tile)
    close(aux, pre_r, what="gelu aux")
    close(out, torch.nn.functional.gelu(pre_r), what="gelu")
    G.gemm(A, B, out, M, N, K, G.KC, G.KC, K, K, N, G.EPI_BF16, bias=bias, resid=res, ldr=N, drop_p=0.1, drop_seed=7,
           tile=tile)
    close(out, res.float() + T.dropout_ref(pre_r, 0.1, 7), what="dropout+resid")
    st = torch.zeros(32, 2, N, device=DEV)
    G.gemm(A, B, out, M, N, K, G.KC, G.KC, K, K, N, G.EPI_BF16, stats=st, tile=tile)
    o = out.float()
    close(st.sum(0)[0], o.sum(0), rtol=1e-3, atol=1e-1, what="stats sum")
    close(st.sum(0)[1], (o * o).sum(0), rtol=1e-3, atol=1e-1, what="stats sumsq")


@pytest.mark.parametrize("tile", TILES)
def test_gemm256_fp32_and_splitk(tile):
    from distributeddeeplearningspark_amd.ops import gemm as G

    # wgrad-shaped: dW[N1,K1] += dy[T,N1]^T x[T,K1] with a long reduction (split-K, atomics)
    T_, N1, K1 = 16384, 768, 3072
    dy, x = rnd(T_, N1, seed=6), rnd(T_, K1, seed=7)
    gw = torch.full((N1, K1), 0.25, device=DEV)
    G.gemm(dy, x, gw, N1, K1, T_, G.RC, G.RC, N1, K1, K1, G.EPI_F32, beta=1.0, tile=tile)
    close(gw, 0.25 + dy.float().T @ x.float(), rtol=1e-3, atol=5e-2, what="split-K fp32 atomics")
    gs = torch.full((N1, K1), 0.25, device=DEV)
    G.gemm(dy, x, gs, N1, K1, T_, G.RC, G.RC, N1, K1, K1, G.EPI_F32, beta=1.0, tile=tile, slabs=True)
    close(gs, 0.25 + dy.float().T @ x.float(), rtol=1e-3, atol=5e-2, what="split-K fp32 slabs")
    M = 4352 if tile == 9 else 512  # persistent: 272 tiles
    out = torch.empty(M, 4096 if tile == 9 else 512, device=DEV)
    A, B = rnd(M, 256, seed=8), rnd(out.shape[1], 256, seed=9)
    G.gemm(A, B, out, M, out.shape[1], 256, G.KC, G.KC, 256, 256, out.shape[1], G.EPI_F32, tile=tile)
    close(out, A.float() @ B.float().T, rtol=1e-3, atol=1e-2, what="fp32 store")


def test_gemm256_auto_selected_for_bert_shapes():
    from distributeddeeplearningspark_amd.ops import gemm as G

    assert G.use_tile256(16384, 16384, 8192, G.KC, G.KC, G.EPI_BF16)
    assert not G.use_tile256(512, 512, 768, G.KC, G.KC, G.EPI_BF16)
    assert not G.use_tile256(16384, 3072, 100, G.KC, G.KC, G.EPI_BF16)


