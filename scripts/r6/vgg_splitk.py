"""VGG-16 (CIFAR shape, batch 256) small-grid 3x3 convolutions run split-K (conv.py splitk_fwd_ok): the
dispatched path (64x64 tiles, fp32 atomics into a workspace + finalize) vs partial slabs on 64x64 and
128x128 tiles at several split counts (+ the finalize summing them).  Interleaved, median us."""
import json
import math
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from distributeddeeplearningspark_amd.ops import conv as CV
from distributeddeeplearningspark_amd.ops import gemm as G
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


def slab(x, w, g, y2, tile, splits):
    K = g.T * g.Ci
    ws = G.splitk_workspace(g.M, g.Co, x.device)
    r = G.gemm(x, w, ws, g.M, g.Co, K, G.KC_GATHER, G.KC, 0, K, g.Co, G.EPI_F32, geom=g.fwd_geom, tile=tile,
               k_split=math.ceil(K / splits / 64) * 64, defer_slabs=True, slabs=True)
    C().splitk_finalize(r[0], y2, g.Co, None, True, None, r[1])


def main():
    for hw, ci, co in ((4, 256, 512), (4, 512, 512), (2, 512, 512)):
        g = CV.geometry(256, hw, hw, ci, co, 3, 3, (1, 1), (1, 1), (1, 1))
        x = (torch.randn(256, hw, hw, ci, device="cuda") * 0.1).to(torch.bfloat16)
        w = (torch.randn(co, 3, 3, ci, device="cuda") * 0.05).to(torch.bfloat16)
        ref = CV.conv_fwd_native(x, w, g, relu=True).float()
        y = torch.empty(256, hw, hw, co, dtype=torch.bfloat16, device="cuda")
        y2 = y.view(g.M, co)
        arms = {"dispatched": lambda: CV.conv_fwd_native(x, w, g, relu=True)}
        t64 = math.ceil(g.M / 64) * math.ceil(co / 64)
        t128 = math.ceil(g.M / 128) * math.ceil(co / 128)
        K = g.T * ci
        for sp in sorted({max(2, min(1024 // t64, K // 512)), max(2, min(768 // t64, K // 512))}):
            arms[f"t3_slab_s{sp}"] = lambda sp=sp: slab(x, w, g, y2, 3, sp)
        for sp in sorted({max(2, min(768 // t128, K // 576)), max(2, min(1536 // t128, K // 576)),
                          max(2, min(1024 // t128, K // 576))}):
            arms[f"t0_slab_s{sp}"] = lambda sp=sp: slab(x, w, g, y2, 0, sp)
        res = {k: [] for k in arms}
        err = {}
        for k, f in arms.items():
            out = f()
            torch.cuda.synchronize()
            got = (out if out is not None else y).float()
            err[k] = round((got - ref).abs().max().item(), 4)
        for _ in range(3):
            for k, f in arms.items():
                res[k].append(timeit(f))
        print(json.dumps({"hw": hw, "ci": ci, "co": co, **{k: [round(statistics.median(v), 1), err[k]]
                                                          for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
