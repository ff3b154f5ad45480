"""Device ETL for the dist-keras column transformers (``csrc/kernels/ingest.hip``).

``etl_device()`` decides where a transformer runs: ``DDL_ETL_DEVICE`` (``cpu`` default,
``cuda`` / ``cuda:N``) or the transformer's own ``device=`` argument.  The GPU path copies
the column to HBM, runs one fp64 kernel and copies the result back — worth it for wide
columns (MNIST pixels, prediction matrices); the numpy path is the reference semantics and
the two agree exactly (same fp64 arithmetic, numpy's first-maximum argmax rule).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ._native import C


def etl_device(explicit=None):
    dev = explicit if explicit is not None else os.environ.get("DDL_ETL_DEVICE", "cpu")
    if dev in (None, "cpu"):
        return None
    dev = torch.device(dev)
    if dev.type != "cuda":
        return None
    if not torch.cuda.is_available():
        raise RuntimeError(f"device ETL requested on {dev} but no GPU is visible")
    return dev


def minmax(v: np.ndarray, o_min: float, scale: float, n_min: float, device) -> np.ndarray:
    """``(v - o_min) * scale + n_min`` in fp64 (the host formula, operation for operation)."""
    x = torch.from_numpy(np.ascontiguousarray(v, dtype=np.float64)).to(device)
    y = torch.empty_like(x)
    C().etl_minmax(x, y, float(o_min), float(scale), float(n_min))
    return y.cpu().numpy()


def one_hot(idx: np.ndarray, K: int, device) -> np.ndarray:
    lab = torch.from_numpy(np.ascontiguousarray(idx, dtype=np.int64)).to(device)
    y = torch.empty((lab.numel(), int(K)), dtype=torch.float64, device=device)
    bad = torch.zeros(1, dtype=torch.int32, device=device)
    C().etl_one_hot(lab, y, bad)
    if int(bad.item()):
        raise ValueError(f"OneHotTransformer: label outside [0, {K})")
    return y.cpu().numpy()


def argmax(v: np.ndarray, device) -> np.ndarray:
    x = torch.from_numpy(np.ascontiguousarray(v, dtype=np.float64)).to(device)
    out = torch.empty(x.shape[0], dtype=torch.int64, device=device)
    C().etl_argmax(x, out)
    return out.cpu().numpy()
