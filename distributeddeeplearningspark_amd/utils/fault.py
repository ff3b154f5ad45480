"""Failure detection and fault injection.

* :class:`Watchdog` — a per-rank heartbeat thread.  The training loop calls ``beat()``
  every step; if no beat arrives within ``timeout_s`` (a hung collective, a dead peer, a
  kernel that never finishes) the watchdog dumps every Python thread's stack and exits
  the process with ``exit_code``.  The launcher (``parallel/launcher.py``) sees the dead
  worker, tears the job down and — with ``max_restarts`` — restarts it; workers resume from
  their last checkpoint (``utils/checkpoint.py``).  RCCL-level errors surface through
  ``TORCH_NCCL_ASYNC_ERROR_HANDLING`` which :func:`enable_async_error_handling` sets.
* :func:`maybe_inject` — deterministic fault injection for tests:
  ``DDL_FAULT_RANK=k DDL_FAULT_STEP=s [DDL_FAULT_MODE=exit|raise|hang]`` makes rank k fail
  at step s of the FIRST attempt only (``DDL_RESTART_COUNT`` = 0), so a restarted job
  completes.
* :func:`replica_checksum` / ``DataParallel.check_replicas`` — divergence detection
  across data-parallel replicas: after a synchronous update every replica
  must hold bit-identical weights.
"""
from __future__ import annotations

import faulthandler
import os
import sys
import threading
import time

import torch


def enable_async_error_handling():
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")


class Watchdog:
    def __init__(self, timeout_s: float = 600.0, exit_code: int = 70, name: str = "ddl-watchdog",
                 on_timeout=None):
        self.timeout_s = float(timeout_s)
        self.exit_code = exit_code
        self.on_timeout = on_timeout
        self._last = time.monotonic()
        self._stop = threading.Event()
        self._step = 0
        self.fired = False
        self._t = threading.Thread(target=self._run, name=name, daemon=True)

    def start(self):
        self._t.start()
        return self

    def beat(self, step: int | None = None):
        self._last = time.monotonic()
        if step is not None:
            self._step = step

    def stop(self):
        self._stop.set()
        if self._t.is_alive():
            self._t.join(timeout=2)

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()

    def _run(self):
        while not self._stop.wait(min(1.0, self.timeout_s / 4)):
            idle = time.monotonic() - self._last
            if idle > self.timeout_s:
                self.fired = True
                sys.stderr.write(f"[ddl-watchdog] no progress for {idle:.0f}s after step {self._step}; "
                                 f"dumping stacks and aborting (exit {self.exit_code})\n")
                faulthandler.dump_traceback(all_threads=True)
                sys.stderr.flush()
                if self.on_timeout is not None:
                    self.on_timeout()
                    return
                os._exit(self.exit_code)


class InjectedFault(RuntimeError):
    pass


def maybe_inject(rank: int, step: int):
    r = os.environ.get("DDL_FAULT_RANK")
    s = os.environ.get("DDL_FAULT_STEP")
    if r is None or s is None or int(os.environ.get("DDL_RESTART_COUNT", "0")) > 0:
        return
    if int(r) != rank or int(s) != step:
        return
    mode = os.environ.get("DDL_FAULT_MODE", "exit")
    sys.stderr.write(f"[ddl-fault] injecting '{mode}' on rank {rank} at step {step}\n")
    sys.stderr.flush()
    if mode == "raise":
        raise InjectedFault(f"injected fault on rank {rank} at step {step}")
    if mode == "hang":
        while True:
            time.sleep(3600)
    os._exit(43)


def replica_checksum(t: torch.Tensor) -> tuple[float, float]:
    """(sum, sum of squares) of a flat fp32 buffer, in float64 — cheap divergence probe."""
    x = t.detach().double()
    return float(x.sum()), float((x * x).sum())
