"""LayerNorm forward / backward at the BERT-base shape (16384 x 768 bf16): microseconds per call
and achieved TB/s (forward moves x + y, backward dy + x + dx), HIP events, median of 5 x 20."""
import json
import os
import statistics
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
    M, H = 16384, 768
    x = torch.randn(M, H, device="cuda").to(torch.bfloat16)
    dy = torch.randn(M, H, device="cuda").to(torch.bfloat16)
    g, b = torch.rand(H, device="cuda") + 0.5, torch.randn(H, device="cuda")
    y, dx = torch.empty_like(x), torch.empty_like(x)
    mean, rstd = torch.empty(M, device="cuda"), torch.empty(M, device="cuda")
    P = C().ln_partial_rows(M)
    ws = torch.empty(P * 2 * H, device="cuda")
    fwd = lambda: C().layernorm_fwd(x, g, b, y, mean, rstd, 1e-12, 0.0, 0)
    bwd = lambda: C().layernorm_bwd(dy, x, mean, rstd, g, dx, None, 0.0, 0, ws, 0.0, 0, 2)
    # the BERT variant: input-gradient dropout in, dropped copy out, 3 partial-sum parts
    dxd = torch.empty_like(x)
    ws3 = torch.empty(P * 3 * H, device="cuda")
    bwd_drop = lambda: C().layernorm_bwd(dy, x, mean, rstd, g, dx, dxd, 0.1, 7, ws3, 0.1, 9, 3)
    fwd_drop = lambda: C().layernorm_fwd(x, g, b, y, mean, rstd, 1e-12, 0.1, 5)
    tf = statistics.median(timeit(fwd) for _ in range(5))
    tb = statistics.median(timeit(bwd) for _ in range(5))
    tfd = statistics.median(timeit(fwd_drop) for _ in range(5))
    tbd = statistics.median(timeit(bwd_drop) for _ in range(5))
    S = x.numel() * 2
    print(json.dumps({"prefetch": os.environ.get("DDL_LN_PREFETCH", "1"), "fwd_us": round(tf, 1),
                      "fwd_TBs": round(2 * S / tf / 1e6, 2), "bwd_us": round(tb, 1), "bwd_TBs": round(3 * S / tb / 1e6, 2),
                      "fwd_dropout_us": round(tfd, 1), "bwd_dropout_parts3_us": round(tbd, 1)}))


if __name__ == "__main__":
    main()
