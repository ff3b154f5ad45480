"""ResNet-50 gathered weight gradients (strided 3x3 and strided 1x1 downsample layers, batch 256): the
dispatched path (conv_wgrad_native: choose_tile + 4 rounds of fp32-atomic split-K) vs 128x128 tiles on
partial slabs at one / two rounds of 3 workgroups per CU.  Interleaved, median us, max |diff|."""
import json
import math
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from distributeddeeplearningspark_amd.ops import conv as CV
from distributeddeeplearningspark_amd.ops import gemm as G

LAYERS = [(14, 512, 512, 3), (28, 256, 256, 3), (56, 128, 128, 3), (14, 1024, 2048, 1), (28, 512, 1024, 1),
          (56, 256, 512, 1)]


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
    for hw, ci, co, k in LAYERS:
        pad = 1 if k == 3 else 0
        g = CV.geometry(256, hw, hw, ci, co, k, k, (2, 2), (pad, pad), (1, 1))
        x = (torch.randn(256, hw, hw, ci, device="cuda") * 0.1).to(torch.bfloat16)
        dy = (torch.randn(256, g.Ho, g.Wo, co, device="cuda") * 0.1).to(torch.bfloat16)
        gw = torch.zeros(co, k, k, ci, device="cuda")
        gw2 = gw.view(co, g.T * ci)
        KK = g.M
        N = g.T * ci
        arms = {"dispatched": lambda: CV.conv_wgrad_native(dy, x, g, gw)}
        t128 = math.ceil(co / 128) * math.ceil(N / 128)
        for rounds in (1, 2):
            sp = max(1, min(rounds * 768 // t128, KK // 1152, 32))
            ks = math.ceil(KK / sp / 64) * 64
            arms[f"slab_r{rounds}_s{math.ceil(KK / ks)}"] = (
                lambda ks=ks: G.gemm(dy, x, gw2, co, N, KK, G.RC, G.RC_GATHER, co, 0, N, G.EPI_F32, beta=1.0,
                                     geom=g.fwd_geom, tile=0, k_split=ks, slabs=True))
        res = {name: [] for name in arms}
        for name, f in arms.items():
            gw.zero_()
            f()
        for _ in range(3):
            for name, f in arms.items():
                res[name].append(timeit(f))
        print(json.dumps({"hw": hw, "ci": ci, "co": co, "k": k, "M": co, "N": N, "K": KK,
                          **{name: round(statistics.median(v), 1) for name, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
