#!/usr/bin/env python
"""Library-path comparison point: a plain PyTorch ResNet-50 (nn.Conv2d/BatchNorm2d,
channels_last, bf16 weights+activations -> MIOpen / hipBLASLt kernels) trained with the
same batch, SGD-momentum and synthetic data as ``bench.py``.  Not part of the framework;
used only to report how the hand-written kernels compare with the vendor libraries.
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import json
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


class Bottleneck(nn.Module):
    def __init__(self, inp, width, stride, down):
        super().__init__()
        out = width * 4
        self.c1, self.b1 = nn.Conv2d(inp, width, 1, bias=False), nn.BatchNorm2d(width)
        self.c2, self.b2 = nn.Conv2d(width, width, 3, stride, 1, bias=False), nn.BatchNorm2d(width)
        self.c3, self.b3 = nn.Conv2d(width, out, 1, bias=False), nn.BatchNorm2d(out)
        self.down = nn.Sequential(nn.Conv2d(inp, out, 1, stride, bias=False), nn.BatchNorm2d(out)) if down else None

    def forward(self, x):
        sc = self.down(x) if self.down is not None else x
        y = F.relu(self.b1(self.c1(x)))
        y = F.relu(self.b2(self.c2(y)))
        return F.relu(self.b3(self.c3(y)) + sc)


class ResNet50(nn.Module):
    def __init__(self, nc=1000):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(),
                                  nn.MaxPool2d(3, 2, 1))
        layers, inp = [], 64
        for si, (nb, w) in enumerate(zip((3, 4, 6, 3), (64, 128, 256, 512))):
            for bi in range(nb):
                layers.append(Bottleneck(inp, w, (1 if si == 0 else 2) if bi == 0 else 1, bi == 0))
                inp = w * 4
        self.layers = nn.Sequential(*layers)
        self.fc = nn.Linear(2048, nc)

    def forward(self, x):
        x = self.layers(self.stem(x))
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    dev = "cuda"
    m = ResNet50().to(dev).to(memory_format=torch.channels_last).to(torch.bfloat16)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
    x = torch.randn(a.batch, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (a.batch,), device=dev)

    def step():
        opt.zero_grad(set_to_none=True)
        loss = F.cross_entropy(m(x).float(), y)
        loss.backward()
        opt.step()
        return loss

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(json.dumps({"impl": "pytorch-miopen-channels_last-bf16", "images_per_sec": round(a.batch * a.steps / dt, 1),
                      "ms_per_step": round(dt / a.steps * 1e3, 2), "batch": a.batch}))


if __name__ == "__main__":
    main()
