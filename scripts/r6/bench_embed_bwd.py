"""BERT-base embedding backward sweeps at T = 16,384 tokens, H = 768: position gradient (sum over the batch) and
token-type partial sums (embed_bwd).  Median us of interleaved rounds."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

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


def main():
    B, S, H = 32, 512, 768
    T = B * S
    de = torch.randn(T, H, device="cuda").to(torch.bfloat16)
    ids = torch.randint(0, 30522, (T,), device="cuda")
    gpos = torch.zeros(512, H, device="cuda")
    P = C().embed_partial_rows(T)
    wsT = torch.empty((P, 2, H), device="cuda")
    arms = {"pos_grad": lambda: C().embed_pos_grad(de, gpos, B, S),
            "type_partials": lambda: C().embed_bwd(ids, None, de, None, None, wsT, 2, S)}
    res = {k: [] for k in arms}
    for _ in range(5):
        for k, f in arms.items():
            res[k].append(timeit(f))
    print(json.dumps({"partial_rows": P, **{k: round(statistics.median(v), 1) for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
