"""BERT MLM head row gather / scatter-sum (layernorm.hip mlm_gather / mlm_scatter) against the PyTorch fp32
reference index_select / index_add, including duplicated and out-of-range positions."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,S,P,H", [(4, 128, 20, 768), (3, 64, 70, 256), (2, 512, 80, 1024)])
def test_mlm_gather_scatter_match_reference(B, S, P, H):
    from distributeddeeplearningspark_amd.ops._native import C

    g = torch.Generator().manual_seed(B * S + P)
    h = torch.randn(B * S, H, generator=g).to(torch.bfloat16).cuda()
    pos = torch.stack([torch.randperm(S, generator=g)[:P] if P <= S else torch.randint(0, S, (P,), generator=g)
                       for _ in range(B)]).cuda()
    pos[0, -3:] = 0  # padding predictions share position 0: their gradients must sum
    pos[1, -1] = S + 5  # out of range: zero row, no gradient
    out = torch.empty(B * P, H, dtype=torch.bfloat16, device="cuda")
    C().mlm_gather(h, pos, out, S)
    flat = (pos + torch.arange(B, device="cuda").view(B, 1) * S).reshape(-1)
    ok = ((pos >= 0) & (pos < S)).reshape(-1)
    ref = torch.where(ok[:, None], h.index_select(0, flat.clamp(0, B * S - 1)), torch.zeros((), dtype=h.dtype,
                                                                                             device="cuda"))
    assert torch.equal(out, ref)
    dout = torch.randn(B * P, H, generator=g).to(torch.bfloat16).cuda()
    dh = torch.full((B * S, H), 7.0, dtype=torch.bfloat16, device="cuda")  # every row must be written
    C().mlm_scatter(dout, pos, dh, S)
    dref = torch.zeros(B * S, H, device="cuda").index_add_(0, flat[ok], dout.float()[ok])
    torch.testing.assert_close(dh.float(), dref, rtol=1e-2, atol=1e-2)
    single = torch.bincount(flat[ok], minlength=B * S) == 1  # single contributions: exact copies
    assert torch.equal(dh[single], dref[single].to(torch.bfloat16))
