"""Fused attention microbenchmark (BERT-base geometry: B=32, H=12, S=512, D=64) with and
without probability dropout; TFLOP/s counts 4*B*H*S^2*D for fwd, 2.5x that for bwd."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributeddeeplearningspark_amd.ops._native import C


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
    B, H, S = 32, 12, 512
    qkv = (torch.randn(B * S, 3 * H * 64, device="cuda") * 0.5).to(torch.bfloat16)
    o = torch.empty(B * S, H * 64, dtype=torch.bfloat16, device="cuda")
    lse = torch.empty(B, H, S, device="cuda")
    do = torch.randn_like(o)
    dvec = torch.empty_like(lse)
    dqkv = torch.empty_like(qkv)
    flop = 4.0 * B * H * S * S * 64
    for p in (0.0, 0.1):
        fwd = lambda: C().attn_fwd(qkv, B, S, H, 0, H * 64, 2 * H * 64, o, lse, None, 0.125, p, 7)  # noqa: E731
        bwd = lambda: C().attn_bwd(qkv, B, S, H, 0, H * 64, 2 * H * 64, o, lse, None, 0.125, p, 7, do, dvec,  # noqa
                                   dqkv)
        fwd()
        tf = [timeit(fwd) for _ in range(3)]
        tb = [timeit(bwd) for _ in range(3)]
        ms_f, ms_b = statistics.median(tf), statistics.median(tb)
        print(json.dumps({"drop_p": p, "fwd_ms": round(ms_f, 4), "fwd_tflops": round(flop / ms_f / 1e9, 1),
                          "bwd_ms": round(ms_b, 4), "bwd_tflops": round(2.5 * flop / ms_b / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
