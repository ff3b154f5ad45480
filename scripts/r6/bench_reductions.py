"""BERT-base gradient reductions, microseconds per call (median of 5 x 20, HIP events): bias_grad over dY
[16384, N] bf16 (the QKV bias: N = 2304; the MLM-head transform: 768), and colsum_partials over the LayerNorm
backward's partial rows [P, 3 x 768]."""
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


out = {}
for N in (2304, 768):
    dy = torch.randn(16384, N, device="cuda").to(torch.bfloat16)
    db = torch.zeros(N, device="cuda")
    us = statistics.median(t(lambda: C().bias_grad(dy, db, N, True)) for _ in range(5))
    ref = dy.float().sum(0)
    db.zero_()
    C().bias_grad(dy, db, N, True)
    torch.cuda.synchronize()
    out[f"bias_grad_16384x{N}_us"] = round(us, 1)
    out[f"bias_grad_16384x{N}_TBs"] = round(dy.numel() * 2 / us / 1e6, 2)
    out[f"bias_grad_16384x{N}_maxrel"] = float(((db - ref).abs().max() / ref.abs().max()).item())
P = C().ln_bwd_rows(16384, 768)
ws = torch.randn(P, 3 * 768, device="cuda")
red = torch.zeros(3 * 768, device="cuda")
out["colsum_rows"] = P
out["colsum_us"] = round(statistics.median(t(lambda: C().colsum_partials(ws, P, 3 * 768, red, True)) for _ in range(5)), 1)
for splits, M_, N_ in ((8, 3072, 768), (8, 2304, 768), (4, 3072, 768)):
    ws8 = torch.randn(splits * M_ * N_, device="cuda")
    c = torch.zeros(M_, N_, device="cuda")
    us = statistics.median(t(lambda: C().slab_reduce(ws8, splits, c, M_, N_, N_, 1.0)) for _ in range(5))
    by = (splits + 2) * M_ * N_ * 4
    out[f"slab_reduce_{splits}x{M_}x{N_}_us"] = round(us, 1)
    out[f"slab_reduce_{splits}x{M_}x{N_}_TBs"] = round(by / us / 1e6, 2)
print(json.dumps(out))
