"""Structured JSONL metrics: one line per logged step with throughput,
step time, per-phase GPU times (from :class:`~.tracing.StepTimer`), all-reduce volume and
achieved bandwidth, and HBM use.  Rank 0 writes by default; every rank can write its own
file (``all_ranks=True``) for straggler analysis."""
from __future__ import annotations

import json
import os
import time

import torch


class MetricsLogger:
    def __init__(self, path: str | None, rank: int = 0, all_ranks: bool = False, every: int = 1):
        self.rank = rank
        self.every = max(1, int(every))
        self.enabled = path is not None and (all_ranks or rank == 0)
        self.path = None
        if self.enabled:
            root, ext = os.path.splitext(path)
            self.path = f"{root}.rank{rank}{ext or '.jsonl'}" if all_ranks else path
            os.makedirs(os.path.dirname(os.path.abspath(self.path)), exist_ok=True)
            self._f = open(self.path, "a", buffering=1)
        self._t_last = time.perf_counter()
        self.records = []

    def log(self, step: int, *, samples: int = 0, loss=None, phases: dict | None = None, comm_bytes: int = 0,
            device=None, **extra):
        now = time.perf_counter()
        dt = now - self._t_last
        self._t_last = now
        if not self.enabled or step % self.every:
            return None
        rec = {"step": step, "time": time.time(), "step_ms": round(dt * 1e3, 3)}
        if samples:
            rec["samples_per_s"] = round(samples / dt, 2) if dt > 0 else None
        if loss is not None:
            rec["loss"] = float(loss)
        if phases:
            rec["phase_ms"] = {k: round(v, 3) for k, v in phases.items()}
            ar = phases.get("allreduce")
            if comm_bytes and ar:
                rec["allreduce_GBps"] = round(comm_bytes / (ar * 1e-3) / 1e9, 2)
        if comm_bytes:
            rec["allreduce_MB"] = round(comm_bytes / 1e6, 3)
        if device is not None and torch.device(device).type == "cuda":
            rec["hbm_alloc_GB"] = round(torch.cuda.memory_allocated(device) / 2**30, 3)
            rec["hbm_peak_GB"] = round(torch.cuda.max_memory_allocated(device) / 2**30, 3)
        rec.update(extra)
        self._f.write(json.dumps(rec) + "\n")
        self.records.append(rec)
        return rec

    def close(self):
        if self.enabled:
            self._f.close()
            self.enabled = False


def read_jsonl(path: str) -> list[dict]:
    with open(path) as f:
        return [json.loads(l) for l in f if l.strip()]
