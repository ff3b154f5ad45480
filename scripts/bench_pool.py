"""Max-pool forward / backward at the ResNet-50 stem shape (256 x 112 x 112 x 64 bf16, 3x3 / 2, pad 1)
and a VGG 2x2 / 2 shape: microseconds per call and achieved TB/s of the bytes each moves."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributeddeeplearningspark_amd.ops._native import C


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
    for N, H, Cc, k, st, p in ((256, 112, 64, 3, 2, 1), (256, 32, 64, 2, 2, 0)):
        Ho = (H + 2 * p - k) // st + 1
        x = torch.randn(N, H, H, Cc, device="cuda").to(torch.bfloat16)
        y = torch.empty(N, Ho, Ho, Cc, dtype=torch.bfloat16, device="cuda")
        am = torch.empty(N, Ho, Ho, Cc, dtype=torch.uint8, device="cuda")
        dy = torch.randn_like(y)
        dx = torch.empty_like(x)
        tf = timeit(lambda: C().maxpool_fwd(x, y, am, k, k, st, st, p, p))
        tb = timeit(lambda: C().maxpool_bwd(dy, am, dx, k, k, st, st, p, p))
        bf = 2 * x.numel() + 2 * y.numel() + am.numel()
        bb = 2 * dy.numel() + am.numel() + 2 * dx.numel()
        print(json.dumps({"shape": [N, H, H, Cc, k, st, p], "fwd_us": round(tf, 1), "fwd_TBs": round(bf / tf / 1e6, 2),
                          "bwd_us": round(tb, 1), "bwd_TBs": round(bb / tb / 1e6, 2)}))


if __name__ == "__main__":
    main()
