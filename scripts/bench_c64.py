"""ResNet-50 stage-1 3x3 conv (batch 256, 56x56, 64 -> 64) forward with BN statistics and its data-
gradient with the fused BN-backward reduce; median ms and TFLOP/s.  DDL_CONV3X3_C64PP=0 selects the
gathered implicit GEMM (the previous path) in a separate process."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributeddeeplearningspark_amd.ops import conv as CV
from distributeddeeplearningspark_amd.ops.norm import SHARDS


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
    for N, H in ((256, 56), (256, 32)):
        C = 64
        g = CV.geometry(N, H, H, C, C, 3, 3, (1, 1), (1, 1), (1, 1))
        x = torch.randn(N, H, H, C, device="cuda").to(torch.bfloat16)
        w = (torch.randn(C, 3, 3, C, device="cuda") * 0.05).to(torch.bfloat16)
        st = torch.zeros((32, 2, C), device="cuda")
        mean, scale, shift = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
        ws = torch.zeros((SHARDS, 2, C), device="cuda")
        bnr = {"x": x, "scale": scale, "shift": shift, "mean": mean, "ws": ws}
        fwd = statistics.median(timeit(lambda: CV.conv_fwd_native(x, w, g, stats=st)) for _ in range(3))
        dgr = statistics.median(timeit(lambda: CV.conv_dgrad_native(x, w, g, bnr=dict(bnr))) for _ in range(3))
        flop = 2.0 * g.M * C * 9 * C
        print(json.dumps({"N": N, "H": H, "c64pp": os.environ.get("DDL_CONV3X3_C64PP", "1"),
                          "fwd": {"ms": round(fwd, 4), "tflops": round(flop / fwd / 1e9, 1)},
                          "dgrad_bnr": {"ms": round(dgr, 4), "tflops": round(flop / dgr / 1e9, 1)}}), flush=True)


if __name__ == "__main__":
    main()
