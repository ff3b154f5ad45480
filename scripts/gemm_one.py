"""Run one GEMM shape on the 128-tile kernel N times (for rocprofv3 PMC passes).
Usage: python scripts/gemm_one.py M N K [a_rc b_rc iters]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributeddeeplearningspark_amd.ops import gemm as G

M, N, K = (int(v) for v in sys.argv[1:4])
a_rc = len(sys.argv) > 4 and sys.argv[4] == "1"
b_rc = len(sys.argv) > 5 and sys.argv[5] == "1"
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 10
a = torch.randn((K, M) if a_rc else (M, K), device="cuda").to(torch.bfloat16)
b = torch.randn((K, N) if b_rc else (N, K), device="cuda").to(torch.bfloat16)
c = torch.empty((M, N), device="cuda", dtype=torch.bfloat16)
for _ in range(iters):
    G.gemm(a, b, c, M, N, K, G.RC if a_rc else G.KC, G.RC if b_rc else G.KC, a.stride(0), b.stride(0), N, G.EPI_BF16,
           tile=0)
torch.cuda.synchronize()
