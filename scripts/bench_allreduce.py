#!/usr/bin/env python
"""RCCL all-reduce micro-benchmark: message-size sweep and bucket-size sweep.

    torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 scripts/bench_allreduce.py
    DDL_FORCE_DIST=1 python scripts/bench_allreduce.py        # N = 1: RCCL's single-rank path

Part 1 (message sweep): one all-reduce of S bytes, S = 1 KB .. 256 MB, fp32 and bf16, timed
with HIP events over ``--iters`` back-to-back calls; reports latency, algorithm bandwidth
(S / t) and bus bandwidth (S / t * 2(N-1)/N, the per-link figure a ring is bound by — compare
with ~153 GB/s per xGMI link).

Part 2 (bucket sweep): the data-parallel engine's actual pattern — a flat gradient of
``--grad-mb`` (ResNet-50 fp32 = 97.5 MB) reduced as ceil(G/b) async bucket all-reduces issued
back to back, b = 1 .. 256 MB.  The bucket size that minimises this time (while staying small
enough to overlap with backward) is the DDL_BUCKET_MB default (parallel/ddp.py).

Rank 0 prints one JSON object per measurement (and ``--out`` writes them all).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.distributed as dist


def _time(fn, iters, warmup):
    for _ in range(warmup):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--max-mb", type=float, default=256)
    ap.add_argument("--grad-mb", type=float, default=97.5, help="flat gradient size for the bucket sweep")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    from distributeddeeplearningspark_amd.parallel import comm

    pg = comm.init_from_env(prefer_gpu=True, force=True)
    assert pg.device.type == "cuda", "bench_allreduce needs a GPU"
    N = pg.world_size
    rows = []

    def emit(d):
        d.update(n_gpus=N, backend=pg.backend)
        rows.append(d)
        if pg.rank == 0:
            print(json.dumps(d), flush=True)

    # ---------------------------------------------------------------- message sweep
    sizes = [1 << 10, 1 << 14, 1 << 16, 1 << 18, 1 << 20]
    mb = 2
    while mb <= args.max_mb:
        sizes.append(int(mb * (1 << 20)))
        mb *= 2
    for dt in (torch.float32, torch.bfloat16):
        es = torch.tensor([], dtype=dt).element_size()
        buf = torch.ones(max(sizes) // es, dtype=dt, device=pg.device)
        for S in sizes:
            v = buf[: S // es]
            it = args.iters if S <= (64 << 20) else max(5, args.iters // 4)
            ms = pg.max_scalar(_time(lambda: dist.all_reduce(v), it, args.warmup))
            alg = S / (ms * 1e-3) / 1e9
            emit({"kind": "message", "dtype": str(dt).split(".")[-1], "bytes": S, "ms": round(ms, 4),
                  "algbw_GBps": round(alg, 1), "busbw_GBps": round(alg * 2 * (N - 1) / N, 1) if N > 1 else None})
        del buf

    # ---------------------------------------------------------------- bucket sweep
    G = int(args.grad_mb * (1 << 20)) // 4
    grad = torch.ones(G, dtype=torch.float32, device=pg.device)
    for bmb in (1, 2, 4, 8, 16, 32, 64, 128, 256):
        step = int(bmb * (1 << 20)) // 4

        def run():
            ws = [dist.all_reduce(grad[i : i + step], async_op=True) for i in range(0, G, step)]
            for w in ws:
                w.wait()

        ms = pg.max_scalar(_time(run, max(5, args.iters // 2), 2))
        emit({"kind": "bucket", "dtype": "float32", "grad_mb": args.grad_mb, "bucket_mb": bmb,
              "buckets": -(-G // step), "ms": round(ms, 4),
              "algbw_GBps": round(G * 4 / (ms * 1e-3) / 1e9, 1)})

    if args.out and pg.rank == 0:
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)
    pg.shutdown()


if __name__ == "__main__":
    main()
