"""ResNet-50 1x1 data-gradients on the streaming kernel (batch 256): plain vs + masked residual vs + fused
BN-backward reduce (mode 3) vs both — time and achieved HBM rate of the bytes each form moves."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from distributeddeeplearningspark_amd.ops import gemm as G
from distributeddeeplearningspark_amd.ops.norm import SHARDS

SHAPES = [(802816, 64, 256), (802816, 256, 64), (802816, 256, 128), (200704, 512, 128), (200704, 512, 256),
          (50176, 1024, 256)]


def timeit(fn, iters=10):
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
    for M, N, K in SHAPES:
        dy = (torch.randn(M, K, device="cuda") * 0.1).to(torch.bfloat16)
        w = (torch.randn(K, N, device="cuda") * 0.1).to(torch.bfloat16)
        r = (torch.randn(M, N, device="cuda") * 0.1).to(torch.bfloat16)
        x = (torch.randn(M, N, device="cuda") * 0.1).to(torch.bfloat16)
        mask = torch.randint(0, 255, (M * N // 8,), dtype=torch.uint8, device="cuda")
        mean = torch.randn(N, device="cuda") * 0.1
        ws = torch.zeros((SHARDS, 2, N), device="cuda")
        out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        bnr = lambda: {"x": x, "mask": mask, "mean": mean, "ws": ws}  # noqa: E731
        arms = {"plain": (lambda: G.linear_dgrad(dy, w, out=out), 2 * (M * K + M * N)),
                "resid": (lambda: G.linear_dgrad(dy, w, out=out, resid=r, resid_mask=mask), 2 * (M * K + 2 * M * N)),
                "bnr": (lambda: G.linear_dgrad(dy, w, out=out, bnr=bnr()), 2 * (M * K + 2 * M * N)),
                "resid_bnr": (lambda: G.linear_dgrad(dy, w, out=out, resid=r, resid_mask=mask, bnr=bnr()),
                              2 * (M * K + 3 * M * N))}
        def nostream(f):
            def g():
                G._USE_STREAM = "0"
                try:
                    return f()
                finally:
                    G._USE_STREAM = "1"
            return g
        for k in list(arms):
            arms["dma_" + k] = (nostream(arms[k][0]), arms[k][1])
        res = {k: [] for k in arms}
        for _ in range(3):
            for k, (f, _) in arms.items():
                res[k].append(timeit(f))
        row = {"M": M, "N": N, "K": K}
        for k, (f, nbytes) in arms.items():
            t = statistics.median(res[k])
            row[k] = [round(t, 1), round(nbytes / t / 1e6, 2)]
        print(json.dumps(row), flush=True)
        del dy, w, r, x, mask, out


if __name__ == "__main__":
    main()
