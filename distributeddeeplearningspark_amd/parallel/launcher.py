"""Worker launcher: the Spark driver -> executor step of the reference, one OS process per
data-parallel worker (one per MI355X on a GPU node).

Three modes, chosen automatically:
  * SPMD  — the job was started by ``torchrun`` (WORLD_SIZE > 1 in the env): every rank
            already runs the driver program; each trains its own partition in-process.
  * local — ``num_workers == 1``: run in the calling process (SingleTrainer, tests).
  * pool  — ``num_workers`` long-lived executor processes (``executors.py``: fresh
            interpreters started as child processes, never an exec of the driver), each
            binding GPU ``rank % n_gpus`` (RCCL) or the CPU (gloo), rendezvousing on a TCP
            store at 127.0.0.1:<free port> once and then serving every training call.
Failures in any worker abort the others and re-raise the worker traceback in the driver
(Spark would retry the task; here a training job is all-or-nothing — see utils/fault.py
for checkpoint-based restart).
"""
from __future__ import annotations

import os
import socket
import time
import traceback


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gpu_count() -> int:
    try:
        import torch

        return torch.cuda.device_count()  # does not initialise the HIP runtime on this image
    except Exception:
        return 0


def workers_per_gpu() -> int:
    """Replicas allowed on one MI355X (``DDL_WORKERS_PER_GPU``, the analog of
    ``spark.executor.cores`` per executor).  Default 1: one worker per GPU."""
    return max(1, int(os.environ.get("DDL_WORKERS_PER_GPU", "1")))


def plan_devices(num_workers: int, device: str | None = None) -> list[str]:
    if device is None:
        device = os.environ.get("DDL_DEVICE", "auto")
    n = _gpu_count()
    if device == "cpu" or (device == "auto" and n == 0):
        return ["cpu"] * num_workers
    wpg = workers_per_gpu()
    if num_workers > n * wpg:
        raise ValueError(f"{num_workers} workers requested but only {n} GPUs x {wpg} workers per GPU: one worker "
                         "per MI355X by default (set DDL_WORKERS_PER_GPU to co-locate small replicas, or pass "
                         "device='cpu' to run the workers on CPU executors)")
    # ranks fill GPUs round-robin so co-located replicas are spread as evenly as possible
    return [f"cuda:{i % n}" for i in range(num_workers)]


def backend_for(devices: list[str]) -> str | None:
    """RCCL needs one rank per GPU; co-located replicas talk over gloo (host-staged)."""
    if devices[0] == "cpu":
        return "gloo"
    return "gloo" if len(set(devices)) < len(devices) else None


def run_workers(fn, num_workers: int, args_per_rank, device: str | None = None, timeout_s: float = 3600.0,
                max_restarts: int | None = None):
    """Run ``fn(rank, world, pg, *args_per_rank[rank])`` on ``num_workers`` workers, return results by rank.

    ``max_restarts`` (default ``DDL_MAX_RESTARTS`` or 0): when a spawned worker dies, all
    workers are torn down and the job is started again (``DDL_RESTART_COUNT`` tells the
    new workers which attempt they are); workers that checkpoint (``utils/checkpoint.py``)
    resume from their last checkpoint — the MI355X analog of Spark re-running a failed task.
    """
    if max_restarts is None:
        max_restarts = int(os.environ.get("DDL_MAX_RESTARTS", "0"))
    attempt = 0
    while True:
        try:
            return _run_once(fn, num_workers, args_per_rank, device, timeout_s, attempt)
        except WorkerFailure as e:
            if attempt >= max_restarts:
                raise
            attempt += 1
            print(f"[ddl-launcher] {e.short}; restarting all workers (attempt {attempt}/{max_restarts})",
                  flush=True)


class WorkerFailure(RuntimeError):
    def __init__(self, msg, short):
        super().__init__(msg)
        self.short = short


def _run_once(fn, num_workers, args_per_rank, device, timeout_s, attempt):
    from . import comm

    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    if env_world > 1:  # SPMD under torchrun
        pg = comm.default_group() or comm.init_from_env()
        if pg.world_size != num_workers:
            raise ValueError(f"torchrun world size {pg.world_size} != num_workers {num_workers}")
        res = fn(pg.rank, pg.world_size, pg, *args_per_rank[pg.rank])
        return pg.all_gather_object(res)
    devices = plan_devices(num_workers, device)
    # DDL_FORCE_POOL=1: a single worker still runs in an executor process (the executor-pool path
    # of the DataFrame bench at N = 1)
    if num_workers == 1 and os.environ.get("DDL_FORCE_POOL", "0") != "1":
        import torch

        dev = torch.device(devices[0])
        if dev.type == "cuda":
            torch.cuda.set_device(dev)
        pg = comm.ProcessGroup(0, 1, 0, dev, None)
        return [fn(0, 1, pg, *args_per_rank[0])]
    # Long-lived executor processes (fresh interpreters started as child processes, never an
    # exec of the driver; reference-style scripts without a __main__ guard work), cached and
    # reused across trainer calls — see executors.py.
    from .executors import ExecutorPool, PoolFailure, get_pool, pooling_enabled

    backend = backend_for(devices)
    pool = get_pool(devices, backend) if pooling_enabled() else ExecutorPool(devices, backend)
    try:
        return pool.run(fn, args_per_rank, timeout_s=timeout_s, attempt=attempt)
    except PoolFailure as e:
        raise WorkerFailure(str(e), e.short) from None
    finally:
        if not pooling_enabled():
            pool.shutdown()


