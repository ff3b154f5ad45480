"""Skinny-K GEMM attribution (ResNet-50 1x1 convs at batch 256): plain vs BN-stats epilogue
vs row-contiguous B (1x1 dgrad) vs hipBLASLt.  Prints one JSON line per shape."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributeddeeplearningspark_amd.ops import gemm as G
from distributeddeeplearningspark_amd.ops.norm import new_stats_workspace

SHAPES = [(802816, 256, 64), (802816, 64, 256), (802816, 64, 64), (802816, 256, 128), (802816, 128, 256),
          (200704, 512, 128), (200704, 128, 512)]


def timeit(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0


def main():
    for M, N, K in SHAPES:
        A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        W = torch.randn(N, K, device="cuda").to(torch.bfloat16)
        Wt = W.T.contiguous()
        out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        stats = new_stats_workspace(N, A.device)
        v = {
            "plain": lambda: G.gemm(A, W, out, M, N, K, G.KC, G.KC, K, K, N, G.EPI_BF16, tile=0),
            "stats": lambda: G.gemm(A, W, out, M, N, K, G.KC, G.KC, K, K, N, G.EPI_BF16, stats=stats, tile=0),
            "rc": lambda: G.gemm(A, Wt, out, M, N, K, G.KC, G.RC, K, N, N, G.EPI_BF16, tile=0),
            "stream": lambda: G.gemm(A, W, out, M, N, K, G.KC, G.KC, K, K, N, G.EPI_BF16, tile=G.TILE_STREAM),
            "stream_stats": lambda: G.gemm(A, W, out, M, N, K, G.KC, G.KC, K, K, N, G.EPI_BF16, stats=stats,
                                           tile=G.TILE_STREAM),
            "stream_rc": lambda: G.gemm(A, Wt, out, M, N, K, G.KC, G.RC, K, N, N, G.EPI_BF16, tile=G.TILE_STREAM),
            "torch": lambda: torch.matmul(A, W.T),
        }
        if not G.stream_panel(N, K):
            for k in [k for k in v if k.startswith("stream")]:
                v.pop(k)
        res = {k: [] for k in v}
        for _ in range(3):
            for k, f in v.items():
                res[k].append(timeit(f))
        gb = (M * K + M * N) * 2 / 1e9
        line = {"M": M, "N": N, "K": K, "min_us_at_6TBs": round(gb / 6e3 * 1e6, 1)}
        line.update({k: round(statistics.median(t), 1) for k, t in res.items()})
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
