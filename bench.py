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
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (resnet50/vgg16 256, bert 32)")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--bucket-mb", type=float, default=None)
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--model", default="resnet50", choices=["resnet50", "vgg16", "bert"],
                    help="resnet50 = the BASELINE headline; vgg16 / bert = the other BASELINE.json DP configs")
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--layers", type=int, default=12)
    args = ap.parse_args()
    if args.model == "vgg16" and args.image == 224:
        args.image = 32
    if args.batch is None:
        args.batch = 32 if args.model == "bert" else 256

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
    if args.model == "bert":
        return bench_bert(args, pg)
    if args.model == "vgg16":
        from distributeddeeplearningspark_amd.models.zoo import vgg16

        n_cls = 10
        model = vgg16(nb_classes=n_cls, input_shape=(args.image, args.image, 3))
    else:
        n_cls = 1000
        model = ResNet50(input_shape=(args.image, args.image, 3), num_classes=n_cls)
    model.compile(SGD(lr=0.1 if args.model == "resnet50" else 0.01, momentum=0.9, weight_decay=5e-5),
                  "sparse_categorical_crossentropy")
    model.place(dev, seed=0)
    ddp = DataParallel(model, pg, bucket_mb=args.bucket_mb, overlap=not args.no_overlap)
    ddp.broadcast_parameters()

    stream = SyntheticImageStream(args.batch, args.image, n_cls, device=dev, seed=rank, n_buffers=4)

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
            "metric": ("images/sec (whole node) ResNet-50 ImageNet-shape at 1/2/4/8 MI355X" if args.model == "resnet50"
                       else "images/sec (whole node) VGG-16 CIFAR-shape"),
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
            "config": {"model": args.model, "global_batch": gb, "seq_len": None, "image": args.image,
                       "per_gpu_batch": args.batch, "parallelism": f"dp{world}", "optimizer": "sgd-momentum",
                       "final_loss": round(lossv, 4)},
        }
        print(json.dumps(out), flush=True)
    pg.shutdown()


def bench_bert(args, pg):
    """BERT-base MLM, seq 512, AdamW; whole-job tokens/sec (synthetic pretraining batches)."""
    from distributeddeeplearningspark_amd.data.synthetic import mlm_batch
    from distributeddeeplearningspark_amd.models.bert import BertConfig, BertForMaskedLM
    from distributeddeeplearningspark_amd.models.optimizers import AdamW
    from distributeddeeplearningspark_amd.parallel.ddp import DataParallel

    rank, world, dev = pg.rank, pg.world_size, pg.device
    cfg = BertConfig(num_hidden_layers=args.layers, max_position_embeddings=max(512, args.seq))
    model = BertForMaskedLM(cfg)
    model.compile(AdamW(lr=1e-4, weight_decay=0.01), "sparse_categorical_crossentropy")
    model.place(dev, seed=0)
    ddp = DataParallel(model, pg, bucket_mb=args.bucket_mb, overlap=not args.no_overlap)
    ddp.broadcast_parameters()
    batches = [mlm_batch(args.batch, args.seq, cfg.vocab_size, seed=rank * 100 + i) for i in range(4)]
    batches = [(model.to_input(x), model.to_target(y)) for x, y in batches]
    it = [0]

    def step():
        x, y = batches[it[0] % len(batches)]
        it[0] += 1
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
    dt_max = pg.max_scalar(time.perf_counter() - t0)
    gb = args.batch * world
    tps = gb * args.seq * args.steps / dt_max
    if rank == 0:
        print(json.dumps({
            "metric": "tokens/sec (whole node) BERT-base MLM seq-len 512",
            "value": round(tps, 1), "unit": "tokens/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt_max * 1000.0 / args.steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
            "config": {"model": "bert-base-mlm" if args.layers == 12 else f"bert-{args.layers}l-mlm",
                       "global_batch": gb, "seq_len": args.seq, "per_gpu_batch": args.batch,
                       "parallelism": f"dp{world}", "optimizer": "adamw", "max_predictions": 80,
                       "sequences_per_sec": round(gb * args.steps / dt_max, 2),
                       "final_loss": round(float(loss), 4)},
        }), flush=True)
    pg.shutdown()


if __name__ == "__main__":
    main()
