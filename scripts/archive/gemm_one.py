"""Run one GEMM shape N times (for rocprofv3 PMC passes).
Usage: python scripts/gemm_one.py M N K [a_rc b_rc iters tile epi]
  tile: 0-3 (128/64 tiles), 4 (256x256 ping-pong), auto;  epi: bf16 (default) | f32 (zeroed fp32 C, split-K
  picked automatically — the weight-gradient form)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributeddeeplearningspark_amd.ops import gemm as G

M, N, K = (int(v) for v in sys.argv[1:4])
a_rc = len(sys.argv) > 4 and sys.argv[4] == "1"
b_rc = len(sys.argv) > 5 and sys.argv[5] == "1"
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 10
tile = sys.argv[7] if len(sys.argv) > 7 else "0"
epi = sys.argv[8] if len(sys.argv) > 8 else "bf16"
tile = None if tile == "auto" else int(tile)
a = torch.randn((K, M) if a_rc else (M, K), device="cuda").to(torch.bfloat16)
b = torch.randn((K, N) if b_rc else (N, K), device="cuda").to(torch.bfloat16)
f32 = epi == "f32"
c = torch.zeros((M, N), device="cuda", dtype=torch.float32 if f32 else torch.bfloat16)
for _ in range(iters):
    G.gemm(a, b, c, M, N, K, G.RC if a_rc else G.KC, G.RC if b_rc else G.KC, a.stride(0), b.stride(0), N,
           G.EPI_F32 if f32 else G.EPI_BF16, beta=1.0 if f32 else 0.0, tile=tile)
torch.cuda.synchronize()
