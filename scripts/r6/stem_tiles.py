"""ResNet-50 stem forward (4x4 conv over the space-to-depth input [256, 115, 115, 16], 64 filters, BN
statistics epilogue): tile shapes of the gathered (GATHER8) implicit GEMM.  Interleaved, median us."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from distributeddeeplearningspark_amd.ops import conv as CV
from distributeddeeplearningspark_amd.ops import gemm as G


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
    N = 256
    xs = (torch.randn(N, 115, 115, 16, device="cuda") * 0.5).to(torch.bfloat16)
    w4 = (torch.randn(64, 4, 4, 16, device="cuda") * 0.1).to(torch.bfloat16)
    g = CV.geometry(N, 115, 115, 16, 64, 4, 4, (1, 1), (0, 0), (1, 1))
    st = torch.zeros(32, 2, 64, device="cuda")
    y = torch.empty(g.M, 64, dtype=torch.bfloat16, device="cuda")
    K = g.T * g.Ci
    am = G.KC_GATHER8 if not g.implicit_fwd else G.KC_GATHER
    arms = {"dispatched": lambda: CV.conv_fwd_native(xs, w4, g, stats=st)}
    for t in (0, 1, 3):
        arms[f"t{t}"] = lambda t=t: G.gemm(xs, w4, y, g.M, 64, K, am, G.KC, 0, K, 64, G.EPI_BF16, geom=g.fwd_geom,
                                           stats=st, tile=t)
    res = {k: [] for k in arms}
    for _ in range(3):
        for k, f in arms.items():
            res[k].append(timeit(f))
    print(json.dumps({"M": g.M, "K": K, "gather8": am == G.KC_GATHER8,
                      **{k: round(statistics.median(v), 1) for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
