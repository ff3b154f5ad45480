"""ResNet-50 7^2 / 14^2 1x1 layers (batch 256) as plain bf16 GEMMs: every tile shape of the 128-row kernel
family and the 256x256 kernel, forward (KC x KC) and data-gradient (KC x RC).  Interleaved, median us."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
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
    return s.elapsed_time(e) / iters * 1e3


def main():
    for hw, n, k in ((7, 2048, 512), (7, 512, 2048), (14, 1024, 256), (14, 256, 1024), (14, 512, 1024)):
        M = 256 * hw * hw
        a = (torch.randn(M, k, device="cuda") * 0.1).to(torch.bfloat16)
        w = (torch.randn(n, k, device="cuda") * 0.1).to(torch.bfloat16)  # [N][K]: forward B
        wr = (torch.randn(k, n, device="cuda") * 0.1).to(torch.bfloat16)  # [K][N]: data-gradient B (RC)
        out = torch.empty(M, n, dtype=torch.bfloat16, device="cuda")
        arms = {"fwd_auto": lambda: G.gemm(a, w, out, M, n, k, G.KC, G.KC, k, k, n, G.EPI_BF16),
                "dg_auto": lambda: G.gemm(a, wr, out, M, n, k, G.KC, G.RC, k, n, n, G.EPI_BF16)}
        for t in (0, 1, 2, 3, G.TILE256):
            arms[f"fwd_t{t}"] = lambda t=t: G.gemm(a, w, out, M, n, k, G.KC, G.KC, k, k, n, G.EPI_BF16, tile=t)
            arms[f"dg_t{t}"] = lambda t=t: G.gemm(a, wr, out, M, n, k, G.KC, G.RC, k, n, n, G.EPI_BF16, tile=t)
        res = {key: [] for key in arms}
        for _ in range(3):
            for key, f in arms.items():
                res[key].append(timeit(f))
        print(json.dumps({"hw": hw, "n": n, "k": k, **{key: round(statistics.median(v), 1) for key, v in res.items()}}),
              flush=True)


if __name__ == "__main__":
    main()
