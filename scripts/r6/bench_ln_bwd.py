"""LayerNorm backward at the BERT-base call (16384 x 768 bf16, parts = 3: [dbias | dgamma | dbeta] partial rows,
output dropout copy, + the column-sum launch that finishes the partial rows): us per call and the HBM rate of the
row sweep (reads dy + x, writes dx + dx_drop = 4 x 25.2 MB).  Median of 5 x 20 calls, HIP events."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from distributeddeeplearningspark_amd.ops._native import C


def t(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


M, H = 16384, 768
x = torch.randn(M, H, device="cuda").to(torch.bfloat16)
dy = torch.randn(M, H, device="cuda").to(torch.bfloat16)
g, b = torch.rand(H, device="cuda") + 0.5, torch.randn(H, device="cuda")
y, dx, dxd = torch.empty_like(x), torch.empty_like(x), torch.empty_like(x)
mean, rstd = torch.empty(M, device="cuda"), torch.empty(M, device="cuda")
C().layernorm_fwd(x, g, b, y, mean, rstd, 1e-12, 0.0, 0)
P = C().ln_bwd_rows(M, H)
ws = torch.empty(P * 3 * H, device="cuda")
red = torch.zeros(3 * H, device="cuda")
bwd = lambda: C().layernorm_bwd(dy, x, mean, rstd, g, dx, dxd, 0.1, 7, ws, 0.0, 0, 3)
col = lambda: C().colsum_partials(ws.view(-1, 3 * H), P, 3 * H, red, True)
copy_src = torch.empty(2 * M * H, dtype=torch.bfloat16, device="cuda")
copy_dst = torch.empty_like(copy_src)
cp = lambda: copy_dst.copy_(copy_src)  # 50 MB read + 50 MB write: the bandwidth reference
tb = statistics.median(t(bwd) for _ in range(5))
tc = statistics.median(t(col) for _ in range(5))
tcp = statistics.median(t(cp) for _ in range(5))
S = M * H * 2
print(json.dumps({"ln_bwd_us": round(tb, 1), "ln_bwd_TBs": round(4 * S / tb / 1e6, 2), "colsum_us": round(tc, 1),
                  "partial_rows": P, "copy_100MB_us": round(tcp, 1), "copy_TBs": round(4 * S / tcp / 1e6, 2)}))
