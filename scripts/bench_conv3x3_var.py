"""Timing of the ResNet-50 3x3 convolution passes (batch 256) for A/B runs of kernel knobs: prints one
JSON line {tag, shape: {fwd_us, dgrad_us, wgrad_us}} with the median of 20 timed launches each.
Usage: DDL_CONV3X3_PRIO=1 python scripts/bench_conv3x3_var.py TAG"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributeddeeplearningspark_amd.ops import conv as CV

PW_SHAPES = [(28, 512, 128), (14, 1024, 256), (14, 256, 1024), (7, 512, 2048), (7, 2048, 512)]
SHAPES = [(56, 64, 1), (56, 128, 2), (28, 128, 1), (28, 256, 2), (14, 256, 1), (14, 512, 2), (7, 512, 1)]


def _time(fn, reps=20):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return round(t[len(t) // 2] * 1000, 1)


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "run"
    N = int(os.environ.get("BATCH", "256"))
    out = {"tag": tag}
    for H, C, s in SHAPES:
        g = CV.geometry(N, H, H, C, C, 3, 3, (s, s), (1, 1), (1, 1))
        x = torch.randn(N, H, H, C, device="cuda").to(torch.bfloat16)
        w = (torch.randn(C, 3, 3, C, device="cuda") * 0.05).to(torch.bfloat16)
        dy = torch.randn(N, g.Ho, g.Wo, C, device="cuda").to(torch.bfloat16)
        gw = torch.zeros(C, 3, 3, C, device="cuda")
        out[f"{H}x{C}s{s}"] = {
            "fwd_us": _time(lambda: CV.conv_fwd_native(x, w, g)),
            "dgrad_us": _time(lambda: CV.conv_dgrad_native(dy, w, g)),
            "wgrad_us": _time(lambda: CV.conv_wgrad_native(dy, x, g, gw)),
        }
        del x, w, dy, gw
    for H, Ci, Co in PW_SHAPES:  # 1x1 weight gradients (split-K fp32 atomics)
        g = CV.geometry(N, H, H, Ci, Co, 1, 1, (1, 1), (0, 0), (1, 1))
        x = torch.randn(N, H, H, Ci, device="cuda").to(torch.bfloat16)
        dy = torch.randn(N, H, H, Co, device="cuda").to(torch.bfloat16)
        gw = torch.zeros(Co, 1, 1, Ci, device="cuda")
        out[f"pw{H}x{Ci}-{Co}"] = {"wgrad_us": _time(lambda: CV.conv_wgrad_native(dy, x, g, gw))}
        del x, dy, gw
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
