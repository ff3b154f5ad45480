#!/usr/bin/env python
"""Headline benchmark (BASELINE.json): ResNet-50, ImageNet-shape, bf16, synthetic data,
images/sec for the WHOLE job across N MI355X (one process per GPU, RCCL over xGMI).

    python bench.py --gpus N --steps K --warmup W
    torchrun --nproc-per-node N bench.py --gpus N ...   (the driver's multi-GPU form)

Each timed step = H2D copy of a pinned uint8 batch on a side stream + fused
normalise kernel + forward + backward (bucketed gradient all-reduce overlapped with
backward when N > 1) + SGD-momentum update of every parameter.  Weak scaling: the
per-GPU batch is fixed, global batch = N * per-GPU batch.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--bucket-mb", type=float, default=None)
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=0)
    args = ap.parse_args()

    from distributeddeeplearningspark_amd.parallel import comm
    from distributeddeeplearningspark_amd.data.ingest import SyntheticImageStream
    from distributeddeeplearningspark_amd.models import ResNet50
    from distributeddeeplearningspark_amd.models.optimizers import SGD
    from distributeddeeplearningspark_amd.parallel.ddp import DataParallel

    pg = comm.init_from_env(prefer_gpu=True)
    rank, world = pg.rank, pg.world_size
    dev = pg.device
    if world != args.gpus and rank == 0:
        print(f"[bench] warning: --gpus {args.gpus} but world size {world}", file=sys.stderr)

    torch.manual_seed(1234 + rank)
    model = ResNet50(input_shape=(args.image, args.image, 3), num_classes=1000)
    model.compile(SGD(lr=0.1, momentum=0.9, weight_decay=5e-5), "sparse_categorical_crossentropy")
    model.place(dev, seed=0)
    ddp = DataParallel(model, pg, bucket_mb=args.bucket_mb, overlap=not args.no_overlap)
    ddp.broadcast_parameters()

    stream = SyntheticImageStream(args.batch, args.image, 1000, device=dev, seed=rank, n_buffers=4)

    def step():
        x, y = stream.next()
        return ddp.train_step(x, y)

    for _ in range(args.warmup):
        step()
    pg.barrier()
    torch.cuda.synchronize(dev) if dev.type == "cuda" else None
    t0 = time.perf_counter()
    loss = None
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize(dev) if dev.type == "cuda" else None
    pg.barrier()
    dt = time.perf_counter() - t0
    dt_max = pg.max_scalar(dt)
    ms = dt_max * 1000.0 / args.steps
    gb = args.batch * world
    ips = gb * args.steps / dt_max
    lossv = float(loss) if loss is not None else float("nan")
    if rank == 0:
        out = {
            "metric": "images/sec (whole node) ResNet-50 ImageNet-shape at 1/2/4/8 MI355X",
            "value": round(ips, 2),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic",
            "config": {"model": "resnet50", "global_batch": gb, "seq_len": None, "image": args.image,
                       "per_gpu_batch": args.batch, "parallelism": f"dp{world}", "optimizer": "sgd-momentum",
                       "final_loss": round(lossv, 4)},
        }
        print(json.dumps(out), flush=True)
    pg.shutdown()


if __name__ == "__main__":
    main()
