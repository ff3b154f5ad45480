"""BatchNorm sweep microbenchmark at the ResNet-50 stage-1 shapes (batch 256): achieved TB/s of
bn_apply (with / without residual + bit mask), bn_bwd_reduce and bn_bwd_dx (modes 2 and 3)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributeddeeplearningspark_amd.ops._native import C


def timeit(fn, reps=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e-3


def main():
    out = []
    for M, Cc, resid in ((802816, 64, False), (802816, 256, True), (200704, 512, True), (50176, 1024, True)):
        x = torch.randn(M, Cc, device="cuda").to(torch.bfloat16)
        dy = torch.randn(M, Cc, device="cuda").to(torch.bfloat16)
        r = torch.randn(M, Cc, device="cuda").to(torch.bfloat16) if resid else None
        sc, sh = torch.rand(Cc, device="cuda") + 0.5, torch.randn(Cc, device="cuda") * 0.1
        mean = torch.randn(Cc, device="cuda") * 0.1
        y = torch.empty_like(x)
        mask = torch.empty(-(-x.numel() // 512) * 64, dtype=torch.uint8, device="cuda") if resid else None
        ws = torch.empty((C().bn_partial_rows(M, Cc), 2, Cc), device="cuda")
        coef = torch.randn(3 * Cc, device="cuda")
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if resid else None
        mode = 3 if resid else 2
        S = x.numel() * 2
        t_apply = timeit(lambda: C().bn_apply(x, sc, sh, r, y, Cc, True, mask))
        t_red = timeit(lambda: C().bn_bwd_reduce(dy, x, mask, sc, sh, mean, ws, Cc, mode))
        t_dx = timeit(lambda: C().bn_bwd_dx(dy, x, mask, sc, sh, coef, dx, dres, Cc, mode))
        row = {"M": M, "C": Cc, "resid": resid,
               "apply_us": round(t_apply * 1e6, 1), "apply_TBs": round((3 if resid else 2) * S / t_apply / 1e12, 2),
               "reduce_us": round(t_red * 1e6, 1), "reduce_TBs": round(2 * S / t_red / 1e12, 2),
               "dx_us": round(t_dx * 1e6, 1), "dx_TBs": round((4 if resid else 3) * S / t_dx / 1e12, 2)}
        t_copy = timeit(lambda: y.copy_(x))  # read + write yardstick at the same size
        row["copy_us"] = round(t_copy * 1e6, 1)
        row["copy_TBs"] = round(2 * S / t_copy / 1e12, 2)
        out.append(row)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
