#!/usr/bin/env python
"""Per-layer A/B of every ResNet-50 convolution shape: our MFMA implicit-GEMM kernels vs
PyTorch's library path (MIOpen, channels_last bf16), forward / data-grad / weight-grad.

Timings interleave the two implementations in one process (rounds x reps, median).
Output: one JSON line per shape + a summary table (gpurun_out/conv_layers.json).
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import json
import statistics
import time

import torch
import torch.nn.functional as F

from distributeddeeplearningspark_amd.ops import conv as CV

# (H, Ci, Co, k, stride) at 224x224 input, batch-independent; count = occurrences in ResNet-50
SHAPES = [
    (224, 3, 64, 7, 2, 1),
    (56, 64, 64, 1, 1, 1), (56, 64, 64, 3, 1, 3), (56, 64, 256, 1, 1, 4), (56, 256, 64, 1, 1, 2),
    (56, 256, 128, 1, 1, 1), (56, 128, 128, 3, 2, 1), (28, 128, 512, 1, 1, 4), (56, 256, 512, 1, 2, 1),
    (28, 512, 128, 1, 1, 3), (28, 128, 128, 3, 1, 3),
    (28, 512, 256, 1, 1, 1), (28, 256, 256, 3, 2, 1), (14, 256, 1024, 1, 1, 6), (28, 512, 1024, 1, 2, 1),
    (14, 1024, 256, 1, 1, 5), (14, 256, 256, 3, 1, 5),
    (14, 1024, 512, 1, 1, 1), (14, 512, 512, 3, 2, 1), (7, 512, 2048, 1, 1, 3), (14, 1024, 2048, 1, 2, 1),
    (7, 2048, 512, 1, 1, 2), (7, 512, 512, 3, 1, 2),
]


def timeit(fn, reps):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default="gpurun_out/conv_layers.json")
    a = ap.parse_args()
    dev = "cuda"
    N = a.batch
    res = []
    tot = {"ours": 0.0, "torch": 0.0}
    for (H, Ci, Co, k, s, cnt) in SHAPES:
        p = k // 2
        x = torch.randn(N, H, H, Ci, device=dev).to(torch.bfloat16)
        w = (torch.randn(Co, k, k, Ci, device=dev) / (k * k * Ci) ** 0.5).to(torch.bfloat16)
        g = CV.geometry(N, H, H, Ci, Co, k, k, (s, s), (p, p), (1, 1))
        dy = torch.randn(N, g.Ho, g.Wo, Co, device=dev).to(torch.bfloat16)
        gw = torch.zeros(Co, k, k, Ci, device=dev)
        xt = x.permute(0, 3, 1, 2)  # channels_last view of NHWC storage
        wt = w.permute(0, 3, 1, 2)
        dyt = dy.permute(0, 3, 1, 2)
        ours = {
            "fwd": lambda: CV.conv_fwd_native(x, w, g),
            "dgrad": lambda: CV.conv_dgrad_native(dy, w, g),
            "wgrad": lambda: CV.conv_wgrad_native(dy, x, g, gw),
        }
        ref = {
            "fwd": lambda: F.conv2d(xt, wt, None, s, p),
            "dgrad": lambda: torch.ops.aten.convolution_backward(dyt, xt, wt, None, [s, s], [p, p], [1, 1], False,
                                                                 [0, 0], 1, [True, False, False]),
            "wgrad": lambda: torch.ops.aten.convolution_backward(dyt, xt, wt, None, [s, s], [p, p], [1, 1], False,
                                                                 [0, 0], 1, [False, True, False]),
        }
        row = {"H": H, "Ci": Ci, "Co": Co, "k": k, "s": s, "count": cnt}
        for ph in ("fwd", "dgrad", "wgrad"):
            if ph == "dgrad" and Ci == 3:
                continue
            o, r = [], []
            for fn in (ours[ph], ref[ph]):
                fn()
            for _ in range(a.rounds):
                o.append(timeit(ours[ph], a.reps))
                r.append(timeit(ref[ph], a.reps))
            mo, mr = statistics.median(o), statistics.median(r)
            flops = 2.0 * N * g.Ho * g.Wo * Co * Ci * k * k
            row[ph] = {"ours_ms": round(mo, 4), "torch_ms": round(mr, 4), "speedup": round(mr / mo, 3),
                       "ours_tflops": round(flops / mo / 1e9, 1)}
            tot["ours"] += mo * cnt
            tot["torch"] += mr * cnt
        res.append(row)
        print(json.dumps(row), flush=True)
    summ = {"batch": N, "sum_ours_ms": round(tot["ours"], 3), "sum_torch_ms": round(tot["torch"], 3),
            "speedup": round(tot["torch"] / tot["ours"], 3)}
    print(json.dumps(summ), flush=True)
    with open(a.out, "w") as f:
        json.dump({"layers": res, "summary": summ}, f, indent=1)


if __name__ == "__main__":
    main()
