"""BERT weight-gradient split-K sweep on the 128x128 partial-slab path (incl. the slab reduce): k_split for
split counts 4..16, vs linear_wgrad as dispatched.  Interleaved rounds, median ms and TF/s per split count."""
import json
import math
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
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
    for name, N, K in (("qkv", 2304, 768), ("ffn1", 3072, 768), ("ffn2", 768, 3072), ("oproj", 768, 768)):
        dy = torch.randn(T, N, device="cuda").to(torch.bfloat16)
        x = torch.randn(T, K, device="cuda").to(torch.bfloat16)
        gw = torch.zeros(N, K, device="cuda")
        arms = {"default": lambda: G.linear_wgrad(dy, x, gw)}
        for sp in (4, 5, 6, 7, 8, 9, 10, 12, 14, 16):
            ks = math.ceil(T / sp / 64) * 64
            arms[f"s{math.ceil(T / ks)}"] = (lambda ks=ks: G.gemm(dy, x, gw, N, K, T, G.RC, G.RC, N, K, K, G.EPI_F32,
                                                                  beta=1.0, tile=0, k_split=ks, slabs=True))
        res = {k: [] for k in arms}
        for _ in range(3):
            for k, f in arms.items():
                res[k].append(timeit(f))
        flop = 2.0 * T * N * K
        print(json.dumps({"shape": name, **{k: round(flop / statistics.median(v) / 1e9, 1) for k, v in res.items()}}),
              flush=True)


if __name__ == "__main__":
    main()
