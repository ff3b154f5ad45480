"""BERT-base weight-gradient GEMMs (dW[N,K] += dy[T,N]^T @ x[T,K], fp32 accumulate, T = 16384
tokens): the RC x RC kernel as dispatched (linear_wgrad), and the same GEMM on K-contiguous
operands (both inputs transposed first; transpose time reported separately).  Median ms, TFLOP/s."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributeddeeplearningspark_amd.ops import gemm as G


def timeit(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    T = 16384
    only = sys.argv[1] if len(sys.argv) > 1 else None  # e.g. "ffn1": one shape, RC kernel only (PMC passes)
    for name, N, K in (("attn_out", 768, 768), ("qkv", 2304, 768), ("ffn1", 3072, 768), ("ffn2", 768, 3072)):
        if only and name != only:
            continue
        if only:
            dy = torch.randn(T, N, device="cuda").to(torch.bfloat16)
            x = torch.randn(T, K, device="cuda").to(torch.bfloat16)
            gw = torch.zeros(N, K, device="cuda")
            for _ in range(10):
                G.linear_wgrad(dy, x, gw)
            torch.cuda.synchronize()
            continue
        dy = torch.randn(T, N, device="cuda").to(torch.bfloat16)
        x = torch.randn(T, K, device="cuda").to(torch.bfloat16)
        gw = torch.zeros(N, K, device="cuda")
        dyt, xt = G.transpose(dy), G.transpose(x)
        res = {"rc": [], "kc": [], "transpose": []}
        for _ in range(5):
            res["rc"].append(timeit(lambda: G.linear_wgrad(dy, x, gw)))
            res["kc"].append(timeit(lambda: G.gemm(dyt, xt, gw, N, K, T, G.KC, G.KC, T, T, K, G.EPI_F32, beta=1.0,
                                                    split_rounds=1)))
            res["transpose"].append(timeit(lambda: (G.transpose(dy), G.transpose(x))))
        flop = 2.0 * T * N * K
        print(json.dumps({"shape": name, **{k: {"ms": round(statistics.median(v), 4),
                                                 "tflops": round(flop / statistics.median(v) / 1e9, 1)}
                                             for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
