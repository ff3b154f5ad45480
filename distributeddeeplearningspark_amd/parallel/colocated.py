"""Device-side commit exchange for dist-keras workers co-located on ONE MI355X.

The reference runs several replicas per executor (``spark.executor.cores = num_processes = 2``,
``ddl_mnist_aztk.py:49-53,66``; ``ddl_nyiso_aztk.py:51-55``).  On a one-GPU box every worker of the
reference's own workloads shares the GPU, and RCCL needs one rank per GPU, so the replicas' process
group is gloo: a commit round used to copy the delta to the host, all-reduce it over local TCP and
copy it back (``comm.py`` host-staged path) — most of the MNIST 8-worker run was spent there.

Here the workers keep the exchange on the GPU:

  * once per training call, each worker allocates a double-buffered fp32 exchange buffer
    ``X[2][n]`` and publishes its IPC handle (torch's CUDA-tensor sharing = hipIpcGetMemHandle /
    dmabuf; ``HSA_ENABLE_IPC_MODE_LEGACY=0`` on this pool) through one ``all_gather_object``; every
    worker maps all its peers' buffers;
  * a round: ``commit_delta`` writes this worker's scaled delta into ``X[parity]`` (HIP) -> device
    synchronize -> ONE host barrier (gloo, no payload) -> ``commit_apply`` sums the peers'
    ``X[parity]`` straight from their HBM into the center and the weights (HIP, one sweep);
  * parity alternates per round: a worker cannot write buffer p again before every peer passed
    the NEXT barrier, by which time each peer has finished reading it (its sum kernel was issued
    before its next device synchronize) — no second barrier per round.

``commit_s`` is split into ``wait_s`` (device synchronize + barrier: waiting for the slowest
co-located peer) and ``xfer_s`` (the sum sweep).  Any failure to map a peer falls back to the
host-staged path with a warning (``available`` is False).
"""
from __future__ import annotations

import time
import warnings

import torch

from ..ops._native import C


def colocated_ok(pg) -> bool:
    """Every rank of the group is on this one GPU (the host-staged gloo group of co-located
    replicas) and the group fits the kernel's peer table.  ``DDL_COLOCATED_EXCHANGE=0`` keeps the
    host-staged path (A/B knob)."""
    import os

    if os.environ.get("DDL_COLOCATED_EXCHANGE", "1") == "0":
        return False
    if not (pg.distributed and pg.host_staged and pg.world_size <= 16):
        return False
    devs = pg.all_gather_object(str(pg.device))
    return len(set(devs)) == 1


class ColocatedExchange:
    def __init__(self, pg, numel: int, device):
        from torch.multiprocessing.reductions import reduce_tensor

        self.pg = pg
        self.n = int(numel)
        self.device = torch.device(device)
        self.parity = 0
        self.wait_s = 0.0
        self.xfer_s = 0.0
        self.available = False
        self.x = torch.zeros((2, self.n), dtype=torch.float32, device=self.device)
        torch.cuda.synchronize(self.device)
        try:
            handle = reduce_tensor(self.x)
            err = None
        except Exception as e:  # sharing unsupported: every rank must learn it
            handle, err = None, f"{type(e).__name__}: {e}"
        allh = pg.all_gather_object((handle, err))
        self.peers = []
        ok = all(h is not None for h, _ in allh)
        if ok:
            try:
                for r, (h, _) in enumerate(allh):
                    if r == pg.rank:
                        self.peers.append(self.x)
                    else:
                        fn, args = h
                        self.peers.append(fn(*args))
            except Exception as e:
                ok, err = False, f"{type(e).__name__}: {e}"
        oks = pg.all_gather_object(ok)
        self.available = all(oks)
        if not self.available:
            self.peers = []
            if pg.rank == 0:
                why = err or next((e for _, e in allh if e), "a peer could not map the buffers")
                warnings.warn(f"co-located device exchange unavailable ({why}); commits stay host-staged",
                              RuntimeWarning, stacklevel=2)

    def commit(self, W: torch.Tensor, center: torch.Tensor, scale: float, elastic: bool, w16=None):
        """One commit round (see module doc).  Returns nothing; ``center`` and ``W`` are updated."""
        p = self.parity
        self.parity ^= 1
        C().commit_delta(W, center, self.x[p], w16 if elastic else None, float(scale), bool(elastic))
        t0 = time.perf_counter()
        torch.cuda.synchronize(self.device)  # my delta is in HBM (and my previous sum is done)
        self.pg.barrier()  # ... and every peer's
        t1 = time.perf_counter()
        C().commit_apply([x[p] for x in self.peers], center, None if elastic else W, None if elastic else w16)
        self.wait_s += t1 - t0
        self.xfer_s += time.perf_counter() - t1

    def close(self):
        """Drop the peer mappings, then a barrier so no worker frees its buffer while mapped."""
        if self.available:
            torch.cuda.synchronize(self.device)
        self.peers = []
        self.pg.barrier()
