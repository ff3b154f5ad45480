"""BERT-base weight-gradient GEMM (RC x RC, fp32 out) configurations: tile x split-K x (slabs | atomics)."""
import math
import os
import sys

sys.path.insert(0, os.getcwd())
import torch

from distributeddeeplearningspark_amd.ops import gemm as G

T = 16384


def timeit(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


for name, N_out, K_in in (("qkv", 2304, 768), ("ffn1", 3072, 768), ("ffn2", 768, 3072), ("oproj", 768, 768)):
    dy = torch.randn(T, N_out, device="cuda").to(torch.bfloat16)
    x = torch.randn(T, K_in, device="cuda").to(torch.bfloat16)
    gw = torch.zeros(N_out, K_in, device="cuda")
    flops = 2.0 * T * N_out * K_in
    ref = (dy.float().t() @ x.float())
    res = {}
    # current dispatch (linear_wgrad)
    ms = timeit(lambda: G.linear_wgrad(dy, x, gw))
    res["default"] = round(flops / ms / 1e9, 1)
    for tile in (0, 1, 2, 3):
        bm, bn = G._TILES[tile]
        tiles = math.ceil(N_out / bm) * math.ceil(K_in / bn)
        for splits in (1, 2, 4, 8, 16):
            ks = math.ceil(T / splits / 64) * 64
            for slabs in (True, False):
                if splits == 1 and not slabs:
                    continue
                def f():
                    G.gemm(dy, x, gw, N_out, K_in, T, G.RC, G.RC, dy.stride(0), x.stride(0), gw.stride(0), G.EPI_F32,
                           beta=1.0, tile=tile, k_split=ks, slabs=slabs)
                try:
                    ms = timeit(f)
                except Exception as e:  # noqa: BLE001
                    continue
                res[f"t{bm}x{bn}/s{splits}/{'slab' if slabs else 'atom'}"] = round(flops / ms / 1e9, 1)
    gw.zero_()
    G.linear_wgrad(dy, x, gw)
    err = ((gw - ref).norm() / ref.norm()).item()
    best = sorted(res.items(), key=lambda kv: -kv[1])[:6]
    print(name, "default", res["default"], "best", best, "rel err", round(err, 5), flush=True)
