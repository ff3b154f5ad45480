"""Synthetic datasets with the reference's shapes (no network: the reference reads
``mnist_train.csv`` / ``NYISO_data_1region_small.csv`` from Azure Blob).

* ``mnist_like``  — ``label`` + 784 pixel columns in 0..250 (``ddl_mnist_aztk.py:113-134``);
  class-dependent blob patterns so a CNN can actually learn them.
* ``nyiso_like``  — hourly ``TimeStamp`` (``MM/DD/YYYY HH:MM:SS`` strings), ``Name``
  (``N.Y.C.``), ``HourAvgLoad`` (MW, daily + weekly seasonality + temperature response)
  and ``temperature`` from 2016-01-02 00:00 (``ddl_nyiso_hdi.ipynb:207``).
* ImageNet / CIFAR / MLM token generators for the north-star benchmarks.
"""
from __future__ import annotations

import datetime as dt

import numpy as np
import pandas as pd


def mnist_like(n: int = 2000, seed: int = 0, num_classes: int = 10, image: int = 28) -> pd.DataFrame:
    rng = np.random.default_rng(seed)
    labels = rng.integers(0, num_classes, n)
    yy, xx = np.mgrid[0:image, 0:image]
    protos = []
    for c in range(num_classes):
        cy, cx = 4 + (c % 5) * (image - 8) / 4, 6 + (c // 5) * (image - 12)
        protos.append(np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / 18.0))
    protos = np.stack(protos)
    imgs = protos[labels] * 220 + rng.normal(0, 12, (n, image, image))
    imgs = np.clip(imgs, 0, 250).round().astype(np.int64)
    data = {"label": labels}
    flat = imgs.reshape(n, -1)
    for i in range(flat.shape[1]):
        data[f"pixel{i}"] = flat[:, i]
    return pd.DataFrame(data)


def nyiso_like(hours: int = 11712, seed: int = 0, start="2016-01-02 00:00:00") -> pd.DataFrame:
    """Default length: 2016-01-02 00:00 through 2017-05-01 23:00 (488 days, 11,712 hours)."""
    rng = np.random.default_rng(seed)
    t0 = dt.datetime.strptime(start, "%Y-%m-%d %H:%M:%S")
    ts = [t0 + dt.timedelta(hours=h) for h in range(hours)]
    h = np.arange(hours)
    hod = h % 24
    dow = (h // 24 + t0.weekday()) % 7
    doy = np.array([t.timetuple().tm_yday for t in ts])
    temp = 55 + 22 * np.sin(2 * np.pi * (doy - 110) / 365.25) + 8 * np.sin(2 * np.pi * (hod - 9) / 24) \
        + rng.normal(0, 3, hours)
    daily = 1 + 0.25 * np.sin(2 * np.pi * (hod - 7) / 24) + 0.1 * np.sin(4 * np.pi * (hod - 3) / 24)
    weekly = np.where(dow >= 5, 0.9, 1.0)
    cool = 1 + 0.012 * np.maximum(temp - 65, 0) + 0.006 * np.maximum(50 - temp, 0)
    load = 5300 * daily * weekly * cool + rng.normal(0, 60, hours)
    return pd.DataFrame({
        "TimeStamp": [t.strftime("%m/%d/%Y %H:%M:%S") for t in ts],
        "Name": ["N.Y.C."] * hours,
        "HourAvgLoad": load.round(1),
        "temperature": temp.round(2),
    })


def imagenet_like(batch: int, image: int = 224, num_classes: int = 1000, seed: int = 0):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 256, (batch, image, image, 3), dtype=np.uint8), rng.integers(0, num_classes, batch)


def cifar_like(n: int, num_classes: int = 10, seed: int = 0):
    rng = np.random.default_rng(seed)
    return rng.normal(0, 1, (n, 32, 32, 3)).astype(np.float32), rng.integers(0, num_classes, n)


def mlm_tokens(batch: int, seq: int = 512, vocab: int = 30522, mask_prob: float = 0.15, seed: int = 0,
               mask_id: int = 103):
    """Random token ids + BERT-style masking: returns (input_ids, labels with -100 on unmasked)."""
    rng = np.random.default_rng(seed)
    ids = rng.integers(1000, vocab, (batch, seq))
    m = rng.random((batch, seq)) < mask_prob
    labels = np.where(m, ids, -100)
    inp = np.where(m, mask_id, ids)
    return inp.astype(np.int64), labels.astype(np.int64)


def mlm_batch(batch: int, seq: int = 512, vocab: int = 30522, max_predictions: int = 80, mask_prob: float = 0.15,
              seed: int = 0, mask_id: int = 103):
    """BERT pretraining-format batch (static shapes, no host sync in the step):
    ``x = {"input_ids"}``, ``y = {"positions" [B,P], "labels" [B,P] (-100 padding), "num_masked"}``.
    Each sequence masks ``min(max_predictions, round(mask_prob*seq))`` positions
    (80/10/10 replacement: [MASK] / random token / unchanged)."""
    rng = np.random.default_rng(seed)
    ids = rng.integers(1000, vocab, (batch, seq)).astype(np.int64)
    n = min(max_predictions, max(1, int(round(mask_prob * seq))))
    pos = np.zeros((batch, max_predictions), np.int64)
    labels = np.full((batch, max_predictions), -100, np.int64)
    inp = ids.copy()
    for b in range(batch):
        p = np.sort(rng.choice(seq, n, replace=False))
        pos[b, :n] = p
        labels[b, :n] = ids[b, p]
        r = rng.random(n)
        inp[b, p[r < 0.8]] = mask_id
        rnd = (r >= 0.8) & (r < 0.9)
        inp[b, p[rnd]] = rng.integers(1000, vocab, int(rnd.sum()))
    return {"input_ids": inp}, {"positions": pos, "labels": labels, "num_masked": batch * n}
