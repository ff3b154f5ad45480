"""Process-group bootstrap: one process per MI355X, ``torch.distributed`` with the
"nccl" backend (= RCCL on ROCm, xGMI peer links), gloo on CPU.

The reference's driver/executor topology (``num_workers = num_executors *
num_processes``, ``ddl_mnist_aztk.py:49-53``) maps to ``world_size`` ranks, one per
GPU; rendezvous goes through torch's TCP store at MASTER_ADDR:MASTER_PORT (the analog
of the dist-keras parameter-server port).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class ProcessGroup:
    rank: int
    world_size: int
    local_rank: int
    device: torch.device
    backend: str | None
    group: object = None
    forced: bool = False  # world-1 group created on purpose (DDL_FORCE_DIST=1): collectives still run

    @property
    def distributed(self) -> bool:
        return self.world_size > 1 or self.forced

    def barrier(self):
        if self.distributed:
            if self.backend == "nccl":
                dist.barrier(group=self.group, device_ids=[self.device.index])
            else:
                dist.barrier(group=self.group)

    @property
    def host_staged(self) -> bool:
        """GPU tensors over gloo (replicas co-located on one GPU): collectives go through host memory."""
        return self.backend == "gloo" and self.device.type == "cuda"

    def all_reduce_(self, t: torch.Tensor, op=dist.ReduceOp.SUM, async_op=False):
        if not self.distributed:
            return None
        if self.host_staged and t.is_cuda:
            h = t.cpu()
            dist.all_reduce(h, op=op, group=self.group)
            t.copy_(h)
            return _DoneWork() if async_op else None
        return dist.all_reduce(t, op=op, group=self.group, async_op=async_op)

    def broadcast_(self, t: torch.Tensor, src: int = 0):
        if not self.distributed:
            return
        if self.host_staged and t.is_cuda:
            h = t.cpu()
            dist.broadcast(h, src, group=self.group)
            t.copy_(h)
            return
        dist.broadcast(t, src, group=self.group)

    def all_gather_object(self, obj):
        if not self.distributed:
            return [obj]
        out = [None] * self.world_size
        dist.all_gather_object(out, obj, group=self.group)
        return out

    def broadcast_object(self, obj, src: int = 0):
        """``obj`` of rank ``src`` on every rank (small picklable objects)."""
        return self.all_gather_object(obj)[src]

    def max_scalar(self, v: float) -> float:
        if not self.distributed:
            return float(v)
        t = torch.tensor([float(v)], dtype=torch.float64, device=self.device if self.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return float(t.item())

    def sum_scalar(self, v: float) -> float:
        if not self.distributed:
            return float(v)
        t = torch.tensor([float(v)], dtype=torch.float64, device=self.device if self.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return float(t.item())

    def shutdown(self):
        if self.distributed and dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:
                pass


class _DoneWork:
    """Completed-work handle for host-staged (synchronous) collectives."""

    def wait(self):
        return True


_DEFAULT: ProcessGroup | None = None


def force_dist_requested() -> bool:
    """``DDL_FORCE_DIST=1``: build a real process group even at world size 1, so the whole
    data-parallel machinery (bucket hooks, RCCL all-reduce / broadcast launches, the
    comm-stream overlap) runs and can be profiled on a single MI355X."""
    return os.environ.get("DDL_FORCE_DIST", "0") == "1"


def init_from_env(prefer_gpu: bool = True, timeout_s: float = 600.0, backend: str | None = None,
                  force: bool | None = None) -> ProcessGroup:
    """Initialise from torchrun-style env (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT).

    ``force`` (default: ``DDL_FORCE_DIST``) creates the "nccl" (RCCL) group — gloo on CPU —
    even when WORLD_SIZE is 1; the single-rank store is an in-process ``HashStore``."""
    global _DEFAULT
    if force is None:
        force = force_dist_requested()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_gpu = prefer_gpu and torch.cuda.is_available()
    if use_gpu:
        n = torch.cuda.device_count()
        idx = local % max(n, 1)
        torch.cuda.set_device(idx)
        device = torch.device("cuda", idx)
    else:
        device = torch.device("cpu")
    be = None
    forced = bool(force) and world == 1
    if world > 1 or forced:
        be = backend or os.environ.get("DDL_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if not dist.is_initialized():
            kw = dict(backend=be, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
            if forced:
                kw["store"] = dist.HashStore()
            if be == "nccl":
                kw["device_id"] = device
            dist.init_process_group(**kw)
    _DEFAULT = ProcessGroup(rank, world, local, device, be, forced=forced)
    return _DEFAULT


def init_process_group(rank: int, world_size: int, master_addr: str = "127.0.0.1", master_port: int = 29500,
                       device: str | torch.device = "cpu", backend: str | None = None,
                       timeout_s: float = 600.0) -> ProcessGroup:
    """Explicit initialisation (used by the Spark-style launcher for its worker processes)."""
    global _DEFAULT
    device = torch.device(device)
    if device.type == "cuda":
        torch.cuda.set_device(device)
    be = None
    if world_size > 1:
        be = backend or ("nccl" if device.type == "cuda" else "gloo")
        if not dist.is_initialized():
            kw = dict(backend=be, init_method=f"tcp://{master_addr}:{master_port}", rank=rank, world_size=world_size,
                      timeout=datetime.timedelta(seconds=timeout_s))
            if be == "nccl":
                kw["device_id"] = device
            dist.init_process_group(**kw)
    _DEFAULT = ProcessGroup(rank, world_size, rank if device.type == "cpu" else (device.index or 0), device, be)
    return _DEFAULT


def default_group() -> ProcessGroup | None:
    return _DEFAULT
