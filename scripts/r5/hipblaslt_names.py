"""torch.matmul (hipBLASLt) on the BERT-base GEMM shapes, for a rocprofv3 kernel trace: the kernel
names encode hipBLASLt's chosen solution (macro tile, wave tile, MFMA, prefetch depth, stream-K)."""
import torch

T = 16384
SHAPES = [("qkv_fwd", T, 2304, 768, False), ("ffn1_fwd", T, 3072, 768, False), ("ffn2_fwd", T, 768, 3072, False),
          ("ffn1_dgrad", T, 768, 3072, True), ("ffn2_dgrad", T, 3072, 768, True), ("sq4096", 4096, 4096, 4096, False)]
for name, M, N, K, rc in SHAPES:
    A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    B = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    Bt = B.T.contiguous() if rc else None
    for _ in range(5):
        C = A @ (Bt if rc else B.T)
    torch.cuda.synchronize()
    print(name, M, N, K, flush=True)
