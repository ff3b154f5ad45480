"""Deterministic-reduction mode (``DDL_DETERMINISTIC=1``).

The fast paths add partial sums from many workgroups with fp32 atomics, whose order (and so the
rounding) changes from run to run: the BatchNorm statistics and backward partial sums that ride in
the GEMM / streaming / halo-conv epilogues (``kStatShards`` atomic shards), split-K weight and data
gradients (``EPI_F32_ATOMIC``), bias and LayerNorm parameter gradients (one atomic per column per
row chunk), the 3x3 weight-gradient slab reduce and the BERT word-embedding gradient (one atomic per
token element).  Under this mode every one of them is replaced by a fixed-order reduction:

  * BN forward statistics: the GEMM epilogues do not accumulate them (``new_stats_workspace`` returns
    None); ``bn_stats`` writes one partial row per workgroup and ``bn_finalize`` sums the rows in index
    order;
  * BN backward partial sums: not fused into the data-gradient epilogues; ``bn_bwd_reduce`` writes
    partial rows (fixed order, as above);
  * split-K: off — every GEMM reduces its whole K inside one workgroup (the split-K workspace paths
    then see one plain fp32 store per element);
  * bias / LayerNorm / column sums and the 3x3 weight-gradient slab reduce: one writer per column
    (the native launchers read the process-wide switch, ``C().set_deterministic``);
  * BERT word-embedding gradient: a stable sort of the token ids, then ONE wave per run of equal ids
    sums the run in token order (``embed_word_grad_det``).

Two runs of the same step on the same inputs then produce bitwise-identical losses and gradient
arenas (``tests/test_gpu_determinism.py``).  Multi-rank runs additionally need fixed all-reduce
bucket boundaries: under this mode ``DataParallel`` skips the timing-based bucket calibration and
uses 32 MB buckets (or an explicit ``DDL_BUCKET_MB``).  The mode costs throughput (more sweeps, fewer
workgroups on the reductions); ``scripts/r4/determinism.sh`` measures the price.  The reference has
no reproducible mode: its parameter server applies commits in arrival order
(``/root/reference/ddl_mnist_aztk.py:216-224``).
"""
from __future__ import annotations

import os
from contextlib import contextmanager

_STATE = {"on": os.environ.get("DDL_DETERMINISTIC", "0") == "1", "native_synced": None}


def enabled() -> bool:
    on = _STATE["on"]
    if _STATE["native_synced"] is not on:
        _sync_native(on)
    return on


def _sync_native(on: bool):
    try:
        from ._native import C, has_native

        if has_native():
            C().set_deterministic(bool(on))
            _STATE["native_synced"] = on
    except Exception:  # no extension (CPU-only tree): the torch paths are deterministic already
        pass


def set_enabled(on: bool):
    """Switch the mode for this process (also the native launchers' switch)."""
    _STATE["on"] = bool(on)
    os.environ["DDL_DETERMINISTIC"] = "1" if on else "0"
    _sync_native(bool(on))


@contextmanager
def deterministic(on: bool = True):
    prev = _STATE["on"]
    set_enabled(on)
    try:
        yield
    finally:
        set_enabled(prev)
