"""ResNet-50 1x1 weight gradients (dW[Co, Ci] += dY^T X over the batch's pixels, batch 256): linear_wgrad as
dispatched vs the 128x128 partial-slab path at several split counts.  Interleaved rounds, median us."""
import json
import math
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from distributeddeeplearningspark_amd.ops import gemm as G

SHAPES = [(64, 64, 56), (256, 64, 56), (64, 256, 56), (128, 256, 56), (512, 128, 28), (128, 512, 28),
          (256, 512, 28), (512, 256, 28), (1024, 256, 14), (256, 1024, 14), (512, 1024, 14), (1024, 512, 14),
          (2048, 512, 7), (512, 2048, 7), (2048, 1024, 7)]


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
    for co, ci, hw in SHAPES:
        T = 256 * hw * hw
        dy = (torch.randn(T, co, device="cuda") * 0.1).to(torch.bfloat16)
        x = (torch.randn(T, ci, device="cuda") * 0.1).to(torch.bfloat16)
        gw = torch.zeros(co, ci, device="cuda")
        arms = {"dispatched": lambda: G.linear_wgrad(dy, x, gw)}
        tiles = math.ceil(co / 128) * math.ceil(ci / 128)
        for sp in sorted({max(1, min(768 // tiles, T // 1152)), max(1, min(1536 // tiles, T // 1152)),
                          max(1, min(384 // tiles, T // 1152))}):
            ks = math.ceil(T / sp / 64) * 64
            arms[f"slab_s{math.ceil(T / ks)}"] = (lambda ks=ks: G.gemm(dy, x, gw, co, ci, T, G.RC, G.RC, co, ci, ci,
                                                                      G.EPI_F32, beta=1.0, tile=0, k_split=ks,
                                                                      slabs=True))
        res = {k: [] for k in arms}
        for _ in range(3):
            for k, f in arms.items():
                res[k].append(timeit(f))
        print(json.dumps({"co": co, "ci": ci, "hw": hw, **{k: round(statistics.median(v), 1) for k, v in res.items()}}),
              flush=True)
        del dy, x, gw


if __name__ == "__main__":
    main()
