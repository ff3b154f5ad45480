"""Cost of the bf16 GEMM epilogue features on BERT-base shapes (random bf16 data): plain (LITE),
+bias+residual, +dropout, +GELU (pre-activation saved), GELU backward.  Median ms and TFLOP/s."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributeddeeplearningspark_amd.ops import gemm as G


def timeit(fn, iters=20):
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
    for name, N, K in (("out_proj", 768, 768), ("ffn1", 3072, 768), ("ffn2", 768, 3072)):
        A = torch.randn(T, K, device="cuda").to(torch.bfloat16)
        W = torch.randn(N, K, device="cuda").to(torch.bfloat16)
        bias = torch.randn(N, device="cuda")
        res = torch.randn(T, N, device="cuda").to(torch.bfloat16)
        aux = torch.empty(T, N, dtype=torch.bfloat16, device="cuda")
        out = torch.empty(T, N, dtype=torch.bfloat16, device="cuda")
        variants = {
            "plain": dict(),
            "bias_resid": dict(bias=bias, resid=res, ldr=N),
            "bias_drop_resid": dict(bias=bias, resid=res, ldr=N, drop_p=0.1, drop_seed=5),
            "bias_gelu": dict(bias=bias, relu=G.ACT_GELU, aux=aux),
            "gelu_bwd": dict(relu=G.ACT_GELU_BWD, aux=aux),
        }
        res_ms = {v: [] for v in variants}
        for _ in range(5):
            for v, kw in variants.items():
                res_ms[v].append(timeit(lambda: G.gemm(A, W, out, T, N, K, G.KC, G.KC, K, K, N, G.EPI_BF16, **kw)))
        flop = 2.0 * T * N * K
        print(json.dumps({"shape": name, **{v: {"ms": round(statistics.median(m), 4),
                                                 "tflops": round(flop / statistics.median(m) / 1e9, 1)}
                                             for v, m in res_ms.items()}}), flush=True)


if __name__ == "__main__":
    main()
