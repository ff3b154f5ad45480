"""ResNet-50 (batch 256) 3x3 stride-1 weight gradients: the halo kernel with fp32 atomics, with partial
slabs + reduce, and the gathered implicit GEMM (DDL_WGRAD3X3=0 path).  Median ms and TFLOP/s per
shape; run under rocprofv3 --kernel-trace --stats for the split between the slab and reduce kernels."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributeddeeplearningspark_amd.ops import conv as CV


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
    N = int(os.environ.get("BATCH", "256"))
    for H, C in ((56, 64), (28, 128), (14, 256), (7, 512)):
        g = CV.geometry(N, H, H, C, C, 3, 3, (1, 1), (1, 1), (1, 1))
        x = torch.randn(N, H, H, C, device="cuda").to(torch.bfloat16)
        dy = torch.randn(N, H, H, C, device="cuda").to(torch.bfloat16)
        gw = torch.zeros(C, 3, 3, C, device="cuda")
        res = {}
        for name, wg3, slab, pp in (("atomic", True, False, False), ("slab", True, True, False),
                                    ("pp_slab", True, True, True), ("pp_atomic", True, False, True),
                                    ("gemm", False, False, False)):
            CV._WG3, CV._WG3_SLAB, CV._WG3_PP = wg3, slab, pp
            res[name] = statistics.median(timeit(lambda: CV.conv_wgrad_native(dy, x, g, gw)) for _ in range(3))
        CV._WG3, CV._WG3_SLAB, CV._WG3_PP = True, True, False
        flop = 2.0 * g.M * C * 9 * C
        print(json.dumps({"H": H, "C": C, **{k: {"ms": round(v, 4), "tflops": round(flop / v / 1e9, 1)}
                                             for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
