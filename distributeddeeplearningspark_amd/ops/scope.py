"""Per-replica workspace scope.

Kernels that keep process-wide scratch per device (the BatchNorm statistics pool in ``norm.py``,
the split-K accumulators in ``gemm.py``) key it by ``(device, scope)``.  The in-process replica group
(``parallel/replicas.py``) runs several model replicas of one GPU concurrently on their own HIP
streams; each replica's step runs under ``replica_scope(r)`` so no two replicas share scratch, and
the weight-gradient side stream (one per device, ``streams.py``) is not used inside a scope.
"""
from __future__ import annotations

from contextlib import contextmanager

_TAG = ""


def tag() -> str:
    return _TAG


@contextmanager
def replica_scope(name):
    global _TAG
    prev, _TAG = _TAG, f"#r{name}"
    try:
        yield
    finally:
        _TAG = prev
