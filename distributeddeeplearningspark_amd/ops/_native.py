"""Loader of the in-tree native extension (``_C.so``: HIP kernels for gfx950 + host runtime).

On a GPU the HIP path is the ONLY path: if the extension is missing or stale an op
raises instead of silently falling back to a PyTorch implementation.  CPU tensors use
the reference implementations in the individual op modules (tests, CPU executors).
``DDL_BACKEND=torch`` forces the reference path on GPU too (A/B benchmarking only).
"""
from __future__ import annotations

import importlib
import os

_C = None
_ERR: Exception | None = None


def _load():
    global _C, _ERR
    if _C is not None or _ERR is not None:
        return
    try:
        _C = importlib.import_module("distributeddeeplearningspark_amd._C")
    except Exception as e:  # pragma: no cover - depends on build state
        _ERR = e
        return
    _warn_if_stale()
    if hasattr(_C, "set_deterministic"):  # the launchers' reduction-order switch (ops/determinism.py)
        from . import determinism

        _C.set_deterministic(determinism._STATE["on"])
        determinism._STATE["native_synced"] = determinism._STATE["on"]


def _warn_if_stale():
    """Loud warning when a kernel/binding source is newer than the loaded extension."""
    import glob
    import warnings

    so = getattr(_C, "__file__", None)
    if not so:
        return
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")
    srcs = [p for pat in ("**/*.hip", "**/*.cpp", "**/*.h") for p in glob.glob(os.path.join(root, pat), recursive=True)]
    try:
        newest = max(os.path.getmtime(p) for p in srcs)
        if newest > os.path.getmtime(so) + 1.0:
            warnings.warn("distributeddeeplearningspark_amd: _C.so is older than its sources; rebuild with "
                          "`python -m distributeddeeplearningspark_amd._build`", RuntimeWarning, stacklevel=3)
    except (ValueError, OSError):
        pass


def has_native() -> bool:
    _load()
    return _C is not None


def C():
    """Return the native module or raise a loud error explaining how to build it."""
    _load()
    if _C is None:
        raise RuntimeError(
            "distributeddeeplearningspark_amd native extension (_C.so) is not available: "
            f"{_ERR!r}. Build it with `python -m distributeddeeplearningspark_amd._build`."
        )
    return _C


def force_reference() -> bool:
    return os.environ.get("DDL_BACKEND", "").lower() == "torch"


def use_native(t) -> bool:
    """True when ``t`` lives on the GPU and the HIP path must be used."""
    if not getattr(t, "is_cuda", False):
        return False
    if force_reference():
        return False
    C()  # raises if missing: no silent fallback on GPU
    return True
