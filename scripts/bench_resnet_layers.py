"""Per-layer roofline table of the ResNet-50 convolutions (batch 256, NHWC bf16).

For every distinct conv shape: forward, data-gradient and weight-gradient time (HIP events,
median of 10), achieved TFLOP/s and GB/s, and the fraction of the roofline bound
max(FLOPs / 2.3 PFLOP/s, bytes / 6 TB/s) reached.  Prints one JSON document."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributeddeeplearningspark_amd.ops import conv as CV
from distributeddeeplearningspark_amd.ops import derived
from distributeddeeplearningspark_amd.ops import gemm as G

PEAK_FLOPS = 2.3e15
PEAK_BW = 6.0e12

# (H_in, Ci, Co, k, stride, count per step) of ResNet-50 v1.5 (stride on the 3x3)
SHAPES = [
    (56, 64, 64, 1, 1, 1), (56, 64, 64, 3, 1, 3), (56, 64, 256, 1, 1, 4), (56, 256, 64, 1, 1, 2),
    (56, 256, 128, 1, 1, 1), (56, 128, 128, 3, 2, 1), (28, 128, 512, 1, 1, 4), (56, 256, 512, 1, 2, 1),
    (28, 512, 128, 1, 1, 3), (28, 128, 128, 3, 1, 3),
    (28, 512, 256, 1, 1, 1), (28, 256, 256, 3, 2, 1), (14, 256, 1024, 1, 1, 6), (28, 512, 1024, 1, 2, 1),
    (14, 1024, 256, 1, 1, 5), (14, 256, 256, 3, 1, 5),
    (14, 1024, 512, 1, 1, 1), (14, 512, 512, 3, 2, 1), (7, 512, 2048, 1, 1, 3), (14, 1024, 2048, 1, 2, 1),
    (7, 2048, 512, 1, 1, 2), (7, 512, 512, 3, 1, 2),
]
# SHAPES=vgg16: the CIFAR VGG-16 convolutions (32x32 input; the 3-channel stem is left out)
VGG16_SHAPES = [
    (32, 64, 64, 3, 1, 1), (16, 64, 128, 3, 1, 1), (16, 128, 128, 3, 1, 1), (8, 128, 256, 3, 1, 1),
    (8, 256, 256, 3, 1, 2), (4, 256, 512, 3, 1, 1), (4, 512, 512, 3, 1, 2), (2, 512, 512, 3, 1, 3),
]
if os.environ.get("SHAPES") == "vgg16":
    SHAPES = VGG16_SHAPES


def timeit(fn, reps=10):
    ts = []
    for _ in range(reps + 2):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts = sorted(ts[2:])
    return ts[len(ts) // 2] * 1e-3


class _Weights:
    """Stand-in for a model whose arena holds ``w``: the derived filter copies (flipped / class / transposed
    weights) then come from one batched launch per call (ops/derived.py), as in a training step, where that
    one launch serves every layer of the model."""

    def __init__(self, w):
        self.arena = type("A", (), {"compute": w})()


def _in_step(m, fn):
    def run():
        derived.begin_step(m)
        try:
            return fn()
        finally:
            derived.end_step()
    return run


def main():
    N = int(os.environ.get("BATCH", "256"))
    rows, total = [], {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0, "bound": 0.0}
    for H, Ci, Co, k, s, cnt in SHAPES:
        p = k // 2
        g = CV.geometry(N, H, H, Ci, Co, k, k, (s, s), (p, p), (1, 1))
        Ho = (H + 2 * p - k) // s + 1
        x = torch.randn(N, H, H, Ci, device="cuda").to(torch.bfloat16)
        w = (torch.randn(Co, k, k, Ci, device="cuda") * 0.05).to(torch.bfloat16)
        dy = torch.randn(N, Ho, Ho, Co, device="cuda").to(torch.bfloat16)
        gw = torch.zeros(Co, k, k, Ci, device="cuda")
        flops = 2.0 * N * Ho * Ho * Co * Ci * k * k
        b_io = 2.0 * x.numel() + 2.0 * dy.numel()
        row = {"H": H, "Ci": Ci, "Co": Co, "k": k, "stride": s, "count": cnt}
        m = _Weights(w)
        dgrad = _in_step(m, lambda: CV.conv_dgrad_native(dy, w, g))
        dg_io = b_io + 2 * w.numel()
        if k == 1 and s == 2:
            # ResNet-50's stride-2 1x1 shortcut (ops/fused_blocks.py, _HALF_RES_SC): the data-gradient is a dense GEMM
            # at half resolution, added at the even pixels by conv1's data-gradient epilogue (rsub) -- no
            # full-resolution tensor of 3/4 zeros is written
            row["dgrad_path"] = "half-resolution GEMM (model path)"
            dgrad = _in_step(m, lambda: G.linear_dgrad(dy.view(-1, Co), w.view(Co, Ci)))
            dg_io = 2.0 * dy.numel() * (1 + Ci / Co) + 2 * w.numel()
        cases = (("fwd", lambda: CV.conv_fwd_native(x, w, g), b_io + 2 * w.numel()),
                 ("dgrad", dgrad, dg_io),
                 ("wgrad", lambda: CV.conv_wgrad_native(dy, x, g, gw), b_io + 4 * w.numel()))
        for name, fn, byts in cases:
            t = timeit(fn)
            bound = max(flops / PEAK_FLOPS, byts / PEAK_BW)
            row[name] = {"ms": round(t * 1e3, 4), "tflops": round(flops / t / 1e12, 1),
                         "gbps": round(byts / t / 1e9, 0), "roofline_frac": round(bound / t, 3)}
            total[name] += t * cnt
            total["bound"] += bound * cnt
        rows.append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)
    total = {k: round(v * 1e3, 3) for k, v in total.items()}
    print(json.dumps({"batch": N, "layers": rows, "total_ms_per_step": total}, indent=1))


if __name__ == "__main__":
    main()
