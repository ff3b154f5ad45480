"""BERT MLM decoder data-gradient dt2[T', 768] = dlogits[T', Vp] @ E[Vp, 768] (T' = 2,560 masked tokens, a
30,528-deep reduction over the padded vocabulary): the dispatched split-K path (64x64 tiles, fp32 atomics
+ finalize) vs 128x128 tiles on partial slabs (+ the finalize summing them), RC weight or a transposed copy.
Interleaved rounds; median us; max |diff| vs the fp32 reference."""
import json
import math
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from distributeddeeplearningspark_amd.ops import gemm as G
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
    return s.elapsed_time(e) / iters * 1e3


def slab_path(dy, w, out, splits, kc):
    M, N = dy.shape
    K = w.shape[1]
    if kc:
        wt = G.transpose(w)
        r = G.gemm(dy, wt, G.splitk_workspace(M, K, dy.device), M, K, N, G.KC, G.KC, dy.stride(0), wt.stride(0), K, G.EPI_F32, tile=0,
                   k_split=math.ceil(N / splits / 64) * 64, defer_slabs=True, slabs=True)
    else:
        r = G.gemm(dy, w, G.splitk_workspace(M, K, dy.device), M, K, N, G.KC, G.RC, dy.stride(0), w.stride(0), K, G.EPI_F32, tile=0,
                   k_split=math.ceil(N / splits / 64) * 64, defer_slabs=True, slabs=True)
    C().splitk_finalize(r[0], out, K, None, False, None, r[1])
    return out


def main():
    T, V, H = 2560, 30528, 768
    dy = (torch.randn(T, V, device="cuda") * 0.05).to(torch.bfloat16)
    w = (torch.randn(V, H, device="cuda") * 0.05).to(torch.bfloat16)
    ref = dy.float() @ w.float()
    out = torch.empty(T, H, dtype=torch.bfloat16, device="cuda")
    arms = {"dispatched": lambda: G.linear_dgrad(dy, w, out=out)}
    for sp in (4, 6, 8, 12):
        arms[f"rc_s{sp}"] = lambda sp=sp: slab_path(dy, w, out, sp, False)
        arms[f"kc_s{sp}"] = lambda sp=sp: slab_path(dy, w, out, sp, True)
    res = {k: [] for k in arms}
    err = {}
    for k, f in arms.items():
        f()
        torch.cuda.synchronize()
        err[k] = round((out.float() - ref).abs().max().item(), 5)
    for _ in range(3):
        for k, f in arms.items():
            res[k].append(timeit(f))
    print(json.dumps({k: [round(statistics.median(v), 1), err[k]] for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
