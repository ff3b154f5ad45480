"""dist-keras trainers (``distkeras.trainers``) on MI355X data parallelism.

Constructor kwargs and the observable surface are the reference's
(``ddl_mnist_aztk.py:216-224``, ``ddl_nyiso_aztk.py:207-218``):
``ADAG(keras_model, worker_optimizer, loss, num_workers, batch_size,
communication_window, num_epoch, features_col, label_col).train(df)`` returns the
trained model; ``trainer.parameter_server.num_updates`` and
``trainer.get_training_time()`` are reported afterwards.

Execution (MI355X-native, not a socket parameter server):
  * ``train(df)`` repartitions the frame into ``num_workers`` shards and starts one
    process per worker (= per GPU, ``parallel/launcher.py``).  Each worker rebuilds the
    model from the serialised ``{'model', 'weights'}`` blob, keeps its shard resident in
    HBM, and trains with its own worker-local optimizer on bf16 HIP kernels.
  * The dist-keras commit/pull protocol becomes a synchronous **periodic delta
    all-reduce over RCCL**: every ``communication_window`` mini-batches all workers
    all-reduce their window-normalised weight delta and continue from the new center
    variable.  ``num_updates`` follows the reference's update law
    ``sum_w floor(num_epoch * floor(rows_w / batch_size) / communication_window)``
    (1425 for the NYISO config); workers that run out of windows keep
    joining the collective with a zero delta so shards of unequal size cannot deadlock.
  * Semantics per algorithm (center c, worker weights W, window k, rank order r):
      ADAG      c += sum_w (W_w - c) / k                       ; W <- c
      DynSGD    c += sum_w (W_w - c) / (s_w + 1)               ; W <- c   (s_w = staleness
                emulated as the number of workers committing before w in the round)
      DOWNPOUR  c += sum_w (W_w - c)                           ; W <- c
      (A)EASGD / EAMSGD  E_w = alpha (W_w - c); W_w -= E_w; c += sum_w E_w   (elastic)
      AveragingTrainer   independent training, c = mean_w W_w at the end
      EnsembleTrainer    independent models, all returned
      SingleTrainer      one worker on the coalesced frame
      SynchronousDataParallel (new)  per-step bucketed gradient all-reduce, overlapped
    These are the synchronous equivalents of dist-keras' asynchronous commits
    (no stale updates are applied in the default ``mode="sync"``).
  * ``mode="sync-grad"``: the per-step gradient all-reduce of ``SynchronousDataParallel``
    (bucketed RCCL, overlapped with backward) under the dist-keras constructor, i.e.
    ``ADAG(..., communication_window=1, mode='sync-grad')``; ``num_updates``
    then counts synchronous steps.
  * ``mode="async"`` (constructor kwarg) reproduces the reference's true asynchrony:
    the driver hosts the native C++ TCP parameter server (``parallel/ps.py``,
    ``csrc/runtime/param_server.cpp``) and workers pull/commit without barriers; DynSGD's
    ``1/(staleness+1)`` scaling is then applied server-side from real staleness.
"""
from __future__ import annotations

import os
import time
import warnings

import numpy as np
import torch

from .models import optimizers as opt_mod
from .parallel.launcher import run_workers
from .utils import deserialize_keras_model, get_states, serialize_keras_model, set_states


# =============================================================================================
#                                    worker side
# =============================================================================================
_INGEST_STREAMS: dict = {}


def ingest_stream(device):
    """ONE side stream per device for every host->HBM shard copy of this process: each extra
    HIP stream can claim a hardware queue, and co-located workers (8 processes on one MI355X)
    oversubscribe the queues if every shard brings its own stream."""
    key = str(device)
    if key not in _INGEST_STREAMS:
        _INGEST_STREAMS[key] = torch.cuda.Stream(device)
    return _INGEST_STREAMS[key]


_SMALL_SHARD = 64 << 20  # below this a direct copy costs less than the stream/event machinery


def _resident(a: np.ndarray, device):
    """Copy a host shard into HBM once, in its own dtype.  Large shards go from pinned memory on
    the ingest side stream (the compute stream waits on an event, the host does not block on
    the transfer); small ones (< 64 MB) are copied directly."""
    t = torch.from_numpy(np.ascontiguousarray(a))
    if device.type != "cuda":
        return t
    if t.numel() * t.element_size() < _SMALL_SHARD:
        return t.to(device)
    pinned = t.pin_memory()
    side = ingest_stream(device)
    with torch.cuda.stream(side):
        d = pinned.to(device, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(side)
    cur = torch.cuda.current_stream(device)
    cur.wait_event(ev)
    d.record_stream(cur)
    return d


class _ShardFeed:
    """How a worker's partition reaches HBM (SURVEY north star: driver-side DataFrame ingest
    streamed from pinned host buffers with hipMemcpyAsync on a side stream, overlapped with
    compute).  Shards keep their column dtype (uint8 pixels stay uint8 on the wire and in HBM)
    and uint8 NHWC images are normalised on the device by ``Model.to_input``.

    * resident — shards up to ``DDL_RESIDENT_MB`` (default 4096 MB; 288 GB of HBM makes this
      the common case): copied once (``_resident``), batches are device slices;
    * stream — ``ingest="stream"`` or larger shards: the native ``BatchLoader``
      (``csrc/runtime/loader.cpp``) fills a ring of pinned buffers on a C++ thread while the
      previous batch trains and ``ShardLoader`` issues each H2D copy on a side stream.

    Trailing partial batches are dropped (dist-keras worker behaviour)."""

    def __init__(self, X, Y, model, cfg):
        self.batch, self.epochs, self.n = int(cfg["batch_size"]), int(cfg["num_epoch"]), int(X.shape[0])
        mode = cfg.get("ingest", "auto")
        if mode not in ("auto", "resident", "stream"):
            raise ValueError(f"ingest={mode!r}: expected 'auto', 'resident' or 'stream'")
        dev = model.device
        limit = float(os.environ.get("DDL_RESIDENT_MB", "4096")) * (1 << 20)
        self.streaming = dev.type == "cuda" and (mode == "stream" or (mode == "auto" and X.nbytes + Y.nbytes > limit))
        if self.streaming:
            from .data.ingest import ShardLoader

            self.loader = ShardLoader(X, Y, self.batch, device=dev, shuffle=False, drop_last=True)
        else:
            self.X, self.Y = _resident(X, dev), _resident(Y, dev)
            if self.X.is_floating_point() and self.X.dtype != model.compute_dtype:
                self.X = self.X.to(model.compute_dtype)  # once, not per batch (labels keep fp32)

    def batches(self):
        bs, nb = self.batch, self.n // self.batch
        for _ in range(self.epochs):
            if self.streaming:
                yield from self.loader  # one epoch per pass over the loader
            else:
                for b in range(nb):
                    yield self.X[b * bs:(b + 1) * bs], self.Y[b * bs:(b + 1) * bs]


def _allreduce_sum(pg, t):
    """In-place sum of a flat fp32 buffer over the workers' group (bucketed, RCCL on GPUs)."""
    if pg.distributed:
        from .parallel.ddp import all_reduce_flat

        all_reduce_flat(pg, t, 64 << 20)


class _Worker:
    def __init__(self, cfg, model, pg, sizes):
        self.cfg, self.model, self.pg, self.sizes = cfg, model, pg, sizes
        bs, E = cfg["batch_size"], cfg["num_epoch"]
        self.k = max(1, int(cfg.get("communication_window", 1)))
        self.steps_all = [E * (s // bs) for s in sizes]
        self.commits_all = [st // self.k for st in self.steps_all]
        self.rounds = max(self.commits_all) if self.commits_all else 0
        self.history: list[float] = []
        self._step = None
        self._hist_dev, self._hist_n = None, 0
        self.commit_s = 0.0  # wall time inside commit rounds (host-side view)

    @property
    def arena(self):
        return self.model.arena

    def batches(self, feed):
        return feed.batches()

    def num_updates(self) -> int:
        return int(sum(self.commits_all))

    # ---------------------------------------------------------------- one mini-batch
    def train_batch(self, xb, yb):
        """One worker-local optimizer step.  On a GPU the step is a replayed hipGraph
        (``models/step.py``) and the loss stays on the device until ``losses()``."""
        if self._step is None:
            from .models.step import CompiledTrainStep

            self._step = CompiledTrainStep(self.model)
        m = self.model
        if m.optimizer.arena is not m.arena:
            m.optimizer.bind(m.arena)
        self._record(self._step(m.to_input(xb), m.to_target(yb)))

    def _record(self, loss):
        if loss.is_cuda:
            if self._hist_dev is None or self._hist_n == self._hist_dev.numel():
                grown = torch.empty(max(1024, 2 * self._hist_n), dtype=torch.float32, device=loss.device)
                if self._hist_dev is not None:
                    grown[: self._hist_n].copy_(self._hist_dev)
                self._hist_dev = grown
            self._hist_dev[self._hist_n].copy_(loss)
            self._hist_n += 1
        else:
            self.history.append(float(loss))

    def losses(self) -> list[float]:
        """Per-batch loss history (one device->host transfer for the whole run)."""
        if self._hist_dev is not None and self._hist_n:
            self.history.extend(self._hist_dev[: self._hist_n].tolist())
            self._hist_n = 0
        return self.history

    def run(self, feed):
        raise NotImplementedError

    # ---------------------------------------------------------------- fault tolerance
    def _tick(self, it):
        from .utils.fault import maybe_inject

        maybe_inject(self.pg.rank, it)
        if getattr(self, "watchdog", None) is not None:
            self.watchdog.beat(it)

    # worker algorithms whose ranks hold state that differs between workers (their own optimizer
    # slots, and for the elastic family their own weights plus the center): checkpointed per rank
    per_rank_state = False

    def _resume(self):
        """(iterations already done, commit rounds already done) from the newest checkpoint;
        per-rank algorithms also get back their own worker state (``self.resumed_extra``)."""
        self.resumed_extra = None
        d = self.cfg.get("checkpoint_dir")
        if not d:
            return 0, 0
        from .utils.checkpoint import latest_checkpoint, load_checkpoint, load_rank_state

        path = latest_checkpoint(d)
        if path is None:
            return 0, 0
        _, meta = load_checkpoint(path, self.model)
        if self.per_rank_state:
            self.resumed_extra = load_rank_state(path, self.model, self.pg.rank)
        ex = meta.get("extra", {})
        self.resumed_from = path
        return int(ex.get("it", 0)), int(ex.get("round", 0))

    def _maybe_checkpoint(self, rnd, it, center=None):
        d, every = self.cfg.get("checkpoint_dir"), int(self.cfg.get("checkpoint_every", 0) or 0)
        if not d or every <= 0 or rnd % every:
            return
        from .utils.checkpoint import save_checkpoint, save_rank_state

        if self.per_rank_state:
            # the center goes to the file in the canonical layout, as the master weights and optimizer slots do
            extra = None if center is None else {"center": self.model.arena.to_canonical(center.detach())}
            save_rank_state(d, self.model, it, self.pg.rank, extra=extra)
            self.pg.barrier()  # every rank file exists before rank 0 publishes `latest`
        save_checkpoint(d, self.model, step=it, extra={"round": rnd, "it": it, "algorithm": self.cfg["algorithm"]},
                        rank=self.pg.rank)
        self.pg.barrier()  # nobody runs ahead of a checkpoint it may have to resume from


class _CommitWorker(_Worker):
    """Periodic commit rounds (ADAG / DynSGD / DOWNPOUR / EASGD family)."""

    rule = "adag"
    per_rank_state = True

    def run(self, feed):
        a = self.arena
        it0, rnd = self._resume()
        ex = self.resumed_extra or {}
        if "center" in ex:  # saved in the canonical layout (_maybe_checkpoint)
            if ex["center"].numel() != a.canon_numel:
                raise ValueError(f"checkpointed center: {ex['center'].numel()} elements, the canonical layout has "
                                 f"{a.canon_numel}")
            center = a.from_canonical(ex["center"].to(a.master.device, torch.float32)).clone()
        else:
            center = a.master.detach().clone()
        self._exchange = None
        if a.master.is_cuda and self.pg.distributed:
            from .parallel.colocated import ColocatedExchange, colocated_ok

            if colocated_ok(self.pg):  # replicas sharing this GPU: device-side exchange (IPC)
                xc = ColocatedExchange(self.pg, a.numel, a.master.device)
                self._exchange = xc if xc.available else None
        it = 0
        try:
            for xb, yb in self.batches(feed):
                it += 1
                if it <= it0:  # resumed: these batches were consumed before the checkpoint
                    continue
                self._tick(it)
                self.train_batch(xb, yb)
                if it % self.k == 0 and rnd < self.rounds:
                    self.commit(center, rnd)
                    rnd += 1
                    self._maybe_checkpoint(rnd, it, center)
            while rnd < self.rounds:  # my shard is exhausted: join the remaining rounds with a zero delta
                self.commit(center, rnd)
                rnd += 1
        finally:
            if self._exchange is not None:
                self.wait_s, self.xfer_s = self._exchange.wait_s, self._exchange.xfer_s
                self._exchange.close()
                self._exchange = None
        return center

    def _contributors(self, rnd):
        return [r for r, c in enumerate(self.commits_all) if rnd < c]

    def commit(self, center, rnd):
        t0 = time.perf_counter()
        try:
            self._commit(center, rnd)
        finally:
            self.commit_s += time.perf_counter() - t0

    def _scale(self, contrib, mine):
        """Per-worker factor of the committed delta (0 for a worker whose shard is exhausted)."""
        if not mine:
            return 0.0
        rule = self.rule
        if rule in ("easgd", "aeasgd", "eamsgd"):
            return float(self.cfg["alpha"])
        if rule == "adag":
            return 1.0 / self.k
        if rule == "dynsgd":
            return 1.0 / (contrib.index(self.pg.rank) + 1)  # staleness = workers committing before me
        return 1.0

    def _commit(self, center, rnd):
        a, pg = self.arena, self.pg
        contrib = self._contributors(rnd)
        mine = pg.rank in contrib
        W = a.master.detach()
        rule = self.rule
        if W.is_cuda:
            # fused HIP commit: X = s (W - center) [W -= X] -> exchange -> center += sum X [W = center]
            elastic = rule in ("easgd", "aeasgd", "eamsgd")
            w16 = None if a.compute is a.master else a.compute
            scale = self._scale(contrib, mine)
            if self._exchange is not None:
                self._exchange.commit(W, center, scale, elastic, w16)
                return
            from .ops._native import C

            if getattr(self, "_xbuf", None) is None or self._xbuf.numel() != W.numel():
                self._xbuf = torch.empty_like(W)
            C().commit_delta(W, center, self._xbuf, w16 if elastic else None, scale, elastic)
            self._allreduce(self._xbuf)
            C().commit_apply([self._xbuf], center, None if elastic else W, None if elastic else w16)
            return
        with torch.no_grad():
            if rule in ("easgd", "aeasgd", "eamsgd"):
                e = (W - center) * self.cfg["alpha"] if mine else torch.zeros_like(W)
                if mine:
                    W.sub_(e)
                self._allreduce(e)
                center.add_(e)
                a.sync_compute()
                return
            d = (W - center) if mine else torch.zeros_like(W)
            if rule == "adag":
                d.div_(self.k)
            elif rule == "dynsgd" and mine:
                staleness = contrib.index(pg.rank)  # workers committing before me in this round
                d.div_(staleness + 1)
            self._allreduce(d)
            center.add_(d)
            W.copy_(center)
            a.sync_compute()

    def _allreduce(self, t):
        _allreduce_sum(self.pg, t)


class _AsyncPSWorker(_Worker):
    """True asynchronous worker against the native parameter server (``mode="async"``):
    pull -> train ``communication_window`` batches -> commit residual -> pull, with no
    barrier between workers (reference ``distkeras/workers.py`` ADAGWorker/DynSGDWorker
    optimize loop).  Rules:
      adag      residual = (W - W_anchor) / window
      dynsgd    residual = (W - W_anchor), the server scales by 1/(staleness+1)
      downpour  residual = (W - W_anchor)
      easgd*    E = alpha * (W - center); W -= E; commit E
    """

    def num_updates(self):
        return self._n

    def run(self, feed):
        from .parallel.ps import ParameterServerClient

        a, algo, k = self.arena, self.cfg["algorithm"], self.k
        W = a.master.detach()
        # the server holds the driver's canonical flat (params.py); the arena may be padded
        cli = ParameterServerClient(self.cfg["ps_port"], self.pg.rank, a.canon_numel)
        self._n = 0
        try:
            def pull():
                with torch.no_grad():
                    a.set_flat(cli.pull())
                return W.clone()

            anchor = pull()
            it = 0
            for xb, yb in self.batches(feed):
                self.train_batch(xb, yb)
                it += 1
                if it % k:
                    continue
                with torch.no_grad():
                    if algo in ("easgd", "aeasgd", "eamsgd"):
                        e = (W - anchor) * self.cfg["alpha"]
                        W.sub_(e)
                        cli.commit(a.to_canonical(e))
                    else:
                        r = W - anchor
                        if algo == "adag":
                            r.div_(k)
                        cli.commit(a.to_canonical(r))
                self._n += 1
                if algo in ("easgd", "aeasgd", "eamsgd"):
                    anchor = a.from_canonical(cli.pull().to(W.device)).clone()  # elastic: keep local weights, refresh center
                    a.sync_compute()
                else:
                    anchor = pull()
        finally:
            cli.close()
        return W.clone()


class _AdagWorker(_CommitWorker):
    rule = "adag"


class _DynSGDWorker(_CommitWorker):
    rule = "dynsgd"


class _DownpourWorker(_CommitWorker):
    rule = "downpour"


class _EASGDWorker(_CommitWorker):
    rule = "easgd"


class _AveragingWorker(_Worker):
    def num_updates(self):
        return 1

    def run(self, feed):
        for xb, yb in self.batches(feed):
            self.train_batch(xb, yb)
        W = self.arena.master.detach()
        with torch.no_grad():
            if self.pg.distributed:
                _allreduce_sum(self.pg, W)
                W.div_(self.pg.world_size)
            self.arena.sync_compute()
        return W.clone()


class _EnsembleWorker(_Worker):
    def num_updates(self):
        return 0

    def run(self, feed):
        for xb, yb in self.batches(feed):
            self.train_batch(xb, yb)
        return self.arena.master.detach().clone()


class _SyncDPWorker(_Worker):
    """Per-step synchronous data parallelism (bucketed RCCL all-reduce overlapped with backward)."""

    def __init__(self, cfg, model, pg, sizes):
        super().__init__(cfg, model, pg, sizes)
        # every replica must take the same number of synchronous steps: shards of unequal size
        # (repartition splits rows to within one) train min(steps) and drop the rest
        self.steps = min(self.steps_all) if self.steps_all else 0
        dropped = max(self.steps_all) - self.steps if self.steps_all else 0
        if dropped and pg.rank == 0:
            warnings.warn(f"SynchronousDataParallel: shards of {sizes} rows give {self.steps_all} steps; every "
                          f"worker trains {self.steps} (up to {dropped} trailing batches dropped on the larger "
                          "shards)", RuntimeWarning, stacklevel=2)
        self.timed_s, self.timed_steps = None, 0

    def num_updates(self):
        return self.steps

    def run(self, feed):
        from .parallel.ddp import DataParallel

        ddp = DataParallel(self.model, self.pg, bucket_mb=self.cfg.get("bucket_mb"))
        it0, _ = self._resume()
        ddp.broadcast_parameters()
        # optional measurement window (bench.py --via-dataframe): steps after `timing_warmup`,
        # bracketed by a barrier + device synchronize on both sides
        tw = self.cfg.get("timing_warmup")
        t0 = None
        it = 0
        for xb, yb in self.batches(feed):
            if it >= self.steps:
                break
            if tw is not None and it == int(tw):
                t0 = self._sync_clock()
            it += 1
            if it <= it0:
                continue
            self._tick(it)
            xb, yb = self.model.to_input(xb), self.model.to_target(yb)
            self._record(ddp.train_step(xb, yb).float())
            self._maybe_checkpoint(it, it)  # every `checkpoint_every` steps (with optimizer state)
        if t0 is not None:
            self.timed_s, self.timed_steps = self._sync_clock() - t0, it - int(tw)
        return self.arena.master.detach().clone()

    def _sync_clock(self):
        if self.model.device.type == "cuda":
            torch.cuda.synchronize(self.model.device)
        self.pg.barrier()
        return time.perf_counter()


_WORKERS = {"adag": _AdagWorker, "dynsgd": _DynSGDWorker, "downpour": _DownpourWorker, "easgd": _EASGDWorker,
            "aeasgd": _EASGDWorker, "eamsgd": _EASGDWorker, "averaging": _AveragingWorker,
            "ensemble": _EnsembleWorker, "single": _EnsembleWorker, "syncdp": _SyncDPWorker}


_MODES = ("sync", "async", "sync-grad")


def _train_worker(rank, world, pg, cfg, blob, X, Y, sizes):
    t0 = time.time()
    model = deserialize_keras_model({k: v for k, v in blob.items() if k not in ("optimizer", "loss")})
    opt = opt_mod.get(cfg["worker_optimizer"])
    if cfg["algorithm"] == "eamsgd" and isinstance(opt, opt_mod.SGD) and not opt.momentum:
        opt.momentum = cfg.get("momentum", 0.9)
    model.compile(opt, cfg["loss"])
    model.seed = cfg.get("seed", 0)
    model.place(pg.device)
    if blob.get("flat") is not None:
        model.arena.set_flat(torch.from_numpy(blob["flat"]))
    if blob.get("states"):
        set_states(model, blob["states"])
    feed = _ShardFeed(X, Y, model, cfg)
    cls = _WORKERS[cfg["algorithm"]]
    if cfg.get("mode") == "async" and issubclass(cls, _CommitWorker):
        cls = _AsyncPSWorker
    elif cfg.get("mode") == "sync-grad":
        cls = _SyncDPWorker
    w = cls(cfg, model, pg, sizes)
    w.watchdog = None
    if cfg.get("watchdog_s"):
        from .utils.fault import Watchdog

        w.watchdog = Watchdog(float(cfg["watchdog_s"])).start()
    try:
        final = w.run(feed)
    finally:
        if w.watchdog is not None:
            w.watchdog.stop()
    if model.device.type == "cuda":
        torch.cuda.synchronize(model.device)
    out = {"rank": rank, "history": w.losses(), "num_updates": w.num_updates(), "time": time.time() - t0,
           "commit_s": w.commit_s, "commit_wait_s": getattr(w, "wait_s", None),
           "commit_xfer_s": getattr(w, "xfer_s", None), "graph": bool(w._step is not None and w._step.captured),
           "ingest": "stream" if feed.streaming else "resident", "timed_s": getattr(w, "timed_s", None),
           "timed_steps": getattr(w, "timed_steps", 0)}
    if rank == 0 or cfg["algorithm"] == "ensemble":
        out["flat"] = model.arena.to_canonical(final).cpu().numpy().copy()
        out["states"] = get_states(model)
    return out


# =============================================================================================
#                                    driver side
# =============================================================================================
class ParameterServer:
    """Facade of the reference's driver-resident parameter server: the center variable
    and the update counter (``trainer.parameter_server.num_updates``)."""

    def __init__(self, model_blob):
        self.model_blob = model_blob
        self.num_updates = 0
        self.center = None
        self.states = None

    def get_model(self):
        m = deserialize_keras_model({k: v for k, v in self.model_blob.items() if k not in ("optimizer", "loss")})
        m.place("cpu")
        if self.center is not None:
            m.arena.set_flat(torch.from_numpy(self.center))
        if self.states:
            set_states(m, self.states)
        return m


class Trainer:
    def __init__(self, keras_model, loss, worker_optimizer, metrics=None, loss_weights=None):
        self.master_model = serialize_keras_model(keras_model)
        self.loss = loss
        self.worker_optimizer = worker_optimizer if not isinstance(worker_optimizer, opt_mod.Optimizer) \
            else worker_optimizer.get_config()
        self.metrics = metrics or ["accuracy"]
        self.loss_weights = loss_weights
        self.history = []
        self.training_time_start = 0.0
        self.training_time_end = 0.0
        self.training_time = 0.0
        self.max_mini_batches_prefetch = 100
        self.parameter_server = ParameterServer(self.master_model)
        self.device = None

    def set_max_prefetch(self, max_mini_batches):
        self.max_mini_batches_prefetch = max_mini_batches

    def record_training_start(self):
        self.training_time = 0.0
        self.training_time_start = time.time()

    def record_training_end(self):
        self.training_time_end = time.time()
        self.training_time = self.training_time_end - self.training_time_start

    def get_training_time(self) -> float:
        return self.training_time

    def get_history(self):
        return self.history

    def get_averaged_history(self):
        from .utils import history_executors_average

        return history_executors_average(self.history)

    def get_executor_history(self, executor_id):
        return self.history[executor_id]

    def train(self, dataframe, shuffle=False):
        raise NotImplementedError


class _ShardedTrainer(Trainer):
    algorithm = "adag"

    def __init__(self, keras_model, worker_optimizer, loss, metrics=None, num_workers=2, batch_size=32,
                 features_col="features", label_col="label", num_epoch=1, communication_window=1,
                 master_port=5000, loss_weights=None, device=None, seed=0, **extra):
        super().__init__(keras_model, loss, worker_optimizer, metrics, loss_weights)
        self.num_workers = int(num_workers)
        self.batch_size = int(batch_size)
        self.features_column = features_col
        self.label_column = label_col
        self.num_epoch = int(num_epoch)
        self.communication_window = int(communication_window)
        self.master_port = master_port
        self.device = device
        self.seed = seed
        mode = extra.get("mode", "sync")
        if mode not in _MODES:
            raise ValueError(f"mode={mode!r}: expected one of {_MODES}")
        if mode == "sync-grad" and self.communication_window != 1:
            warnings.warn(f"mode='sync-grad' all-reduces gradients every step: communication_window="
                          f"{self.communication_window} is ignored", RuntimeWarning, stacklevel=3)
        self.extra = extra

    def _cfg(self):
        return {"algorithm": self.algorithm, "worker_optimizer": self.worker_optimizer, "loss": self.loss,
                "batch_size": self.batch_size, "num_epoch": self.num_epoch,
                "communication_window": self.communication_window, "seed": self.seed, **self.extra}

    def _shards(self, dataframe, shuffle):
        df = dataframe
        if shuffle:
            from .utils import shuffle as _shuffle

            df = _shuffle(df, self.seed)
        if df.rdd_partitions_count() != self.num_workers:
            df = df.repartition(self.num_workers)
        # column dtypes are kept (uint8 pixels stay uint8; float64 narrows to float32)
        parts = df.partition_arrays([self.features_column, self.label_column], None)
        return [p[0] for p in parts], [p[1] for p in parts]

    def train(self, dataframe, shuffle=False):
        self.record_training_start()
        Xs, Ys = self._shards(dataframe, shuffle)
        sizes = [x.shape[0] for x in Xs]
        self.worker_rows = list(sizes)
        cfg = self._cfg()
        server = None
        if cfg.get("mode") == "async" and issubclass(_WORKERS[self.algorithm], _CommitWorker):
            server = self._start_async_server(cfg)
        try:
            devices = self._replica_devices(cfg, server, Xs, Ys)
            if devices is not None:
                results = self._train_replica_groups(cfg, Xs, Ys, sizes, devices)
            else:
                args = [(cfg, self.master_model, Xs[r], Ys[r], sizes) for r in range(self.num_workers)]
                results = run_workers(_train_worker, self.num_workers, args, device=self.device,
                                      max_restarts=self.extra.get("max_restarts"))
        finally:
            if server is not None:
                center, n_upd = server.center().numpy().copy(), server.num_updates
                server.stop()
        self.history = [r["history"] for r in results]
        ps = self.parameter_server
        if server is not None:  # the driver-hosted center is the trained model
            ps.num_updates, ps.center = int(n_upd), center
        else:
            ps.num_updates = int(results[0]["num_updates"])
            ps.center = results[0]["flat"]
        ps.states = results[0].get("states")
        self.worker_times = [r["time"] for r in results]
        self.worker_commit_times = [r.get("commit_s", 0.0) for r in results]
        self._results = results
        model = ps.get_model()
        self.record_training_end()
        return model

    def _replica_devices(self, cfg, server, Xs=None, Ys=None):
        """The worker -> device plan when the co-located workers run as in-process replica groups
        (``parallel/replicas.py``), else None (one OS process per worker).

        Replica groups keep every shard resident in HBM, so they are used only when the user did
        not ask for streamed ingest (``ingest="stream"``) and each group's shards together fit the
        resident limit (``DDL_RESIDENT_MB``, as ``_ShardFeed`` applies per worker); otherwise the
        process-per-worker path streams the shards through the pinned ring."""
        from .parallel import replicas as _rep
        from .parallel.launcher import plan_devices

        if server is not None or self.num_workers < 2:
            return None
        if cfg.get("checkpoint_dir") or cfg.get("watchdog_s") or self.extra.get("max_restarts"):
            return None  # per-rank checkpoints / watchdog / restart live on the process-per-worker path
        if cfg.get("ingest", "auto") == "stream":
            return None
        world = int(os.environ.get("WORLD_SIZE", "1"))
        if world > 1:
            # torchrun SPMD with more workers than ranks (the reference's 2 processes per executor on one
            # process per GPU): rank r hosts workers r*k .. r*k + k - 1 as one replica group; the groups'
            # commit sums meet over the job's process group.  num_workers == WORLD_SIZE keeps one worker
            # per rank (process-per-worker SPMD).
            if self.num_workers <= world or self.num_workers % world:
                return None
            k = self.num_workers // world
            devices = [f"rank{w // k}" for w in range(self.num_workers)]
            return devices if _rep.applies(cfg, devices) else None
        devices = plan_devices(self.num_workers, self.device)
        if not _rep.applies(cfg, devices):
            return None
        if Xs is not None and devices[0] != "cpu":
            limit = float(os.environ.get("DDL_RESIDENT_MB", "4096")) * (1 << 20)
            for g in _rep.plan(devices):
                if sum(Xs[r].nbytes + Ys[r].nbytes for r in g) > limit:
                    return None
        return devices

    def _train_replica_groups(self, cfg, Xs, Ys, sizes, devices):
        from .parallel import comm
        from .parallel import replicas as _rep

        groups = _rep.plan(devices)
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:  # torchrun: this rank's group, results gathered
            pg = comm.default_group() or comm.init_from_env()
            if len(groups) != pg.world_size:
                raise ValueError(f"{len(groups)} replica groups for torchrun world size {pg.world_size}")
            g = groups[pg.rank]
            res = _rep.train_group(pg.rank, pg.world_size, pg, cfg, self.master_model, [Xs[r] for r in g],
                                   [Ys[r] for r in g], g, sizes)
            res = [x for grp in pg.all_gather_object(res) for x in grp]
        elif len(groups) == 1:  # one device: the replicas train in this process (no executor hop)
            g = groups[0]
            dev = torch.device(devices[g[0]])
            if dev.type == "cuda":
                torch.cuda.set_device(dev)
            pg = comm.ProcessGroup(0, 1, 0, dev, None)
            res = _rep.train_group(0, 1, pg, cfg, self.master_model, [Xs[r] for r in g], [Ys[r] for r in g], g, sizes)
        else:  # one executor process per device, partial sums all-reduced over RCCL (gloo on CPU)
            args = [(cfg, self.master_model, [Xs[r] for r in g], [Ys[r] for r in g], g, sizes) for g in groups]
            per = run_workers(_rep.train_group, len(groups), args, device="cpu" if devices[0] == "cpu" else self.device)
            res = [x for grp in per for x in grp]
        return sorted(res, key=lambda r: r["rank"])


    def _start_async_server(self, cfg):
        """Host the native parameter server on the driver (single node, 127.0.0.1)."""
        import os

        from .parallel.ps import RULE_ADD, RULE_DYNSGD, ParameterServerProcess

        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            raise NotImplementedError("mode='async' runs workers from the driver; under torchrun use mode='sync'")
        blob = {k: v for k, v in self.master_model.items() if k not in ("optimizer", "loss")}
        m = deserialize_keras_model(blob, device="cpu")
        rule = RULE_DYNSGD if self.algorithm == "dynsgd" else RULE_ADD
        server = ParameterServerProcess(m.arena.master.detach(), rule=rule,
                                        port=int(self.extra.get("ps_port", 0)))
        cfg["ps_port"] = server.port
        return server


class SingleTrainer(_ShardedTrainer):
    """One worker on the coalesced frame (``ddl_mnist_aztk.py:215``)."""

    algorithm = "single"

    def __init__(self, keras_model, worker_optimizer, loss, metrics=None, features_col="features",
                 label_col="label", num_epoch=1, batch_size=32, **kw):
        super().__init__(keras_model, worker_optimizer, loss, metrics, 1, batch_size, features_col, label_col,
                         num_epoch, 1, **kw)

    def train(self, dataframe, shuffle=False):
        model = super().train(dataframe.coalesce(1), shuffle)
        self.parameter_server.num_updates = len(self.history[0]) if self.history else 0
        return model


class AveragingTrainer(_ShardedTrainer):
    algorithm = "averaging"

    def __init__(self, keras_model, worker_optimizer, loss, metrics=None, features_col="features",
                 label_col="label", num_epoch=1, batch_size=32, num_workers=2, **kw):
        super().__init__(keras_model, worker_optimizer, loss, metrics, num_workers, batch_size, features_col,
                         label_col, num_epoch, 1, **kw)


class EnsembleTrainer(_ShardedTrainer):
    algorithm = "ensemble"

    def __init__(self, keras_model, worker_optimizer, loss, metrics=None, features_col="features",
                 label_col="label", batch_size=32, num_ensembles=2, num_epoch=1, **kw):
        super().__init__(keras_model, worker_optimizer, loss, metrics, num_ensembles, batch_size, features_col,
                         label_col, num_epoch, 1, **kw)

    def train(self, dataframe, shuffle=False):
        super().train(dataframe, shuffle)
        models = []
        for r in self._results:
            ps = ParameterServer(self.master_model)
            ps.center, ps.states = r["flat"], r.get("states")
            models.append(ps.get_model())
        return models


class DistributedTrainer(_ShardedTrainer):
    pass


class AsynchronousDistributedTrainer(DistributedTrainer):
    def __init__(self, *a, parallelism_factor=1, **kw):
        super().__init__(*a, **kw)
        self.parallelism_factor = parallelism_factor


class ADAG(AsynchronousDistributedTrainer):
    """Asynchronous Distributed Adaptive Gradients — window-normalised delta commits."""

    algorithm = "adag"

    def __init__(self, keras_model, worker_optimizer, loss, metrics=None, num_workers=2, batch_size=32,
                 features_col="features", label_col="label", num_epoch=1, communication_window=12,
                 master_port=5000, loss_weights=None, **kw):
        super().__init__(keras_model, worker_optimizer, loss, metrics, num_workers, batch_size, features_col,
                         label_col, num_epoch, communication_window, master_port, loss_weights, **kw)


class DynSGD(AsynchronousDistributedTrainer):
    """Staleness-aware async SGD (commit scaled by 1/(staleness+1))."""

    algorithm = "dynsgd"

    def __init__(self, keras_model, worker_optimizer, loss, metrics=None, num_workers=2, batch_size=32,
                 features_col="features", label_col="label", num_epoch=1, communication_window=5,
                 master_port=5000, loss_weights=None, **kw):
        super().__init__(keras_model, worker_optimizer, loss, metrics, num_workers, batch_size, features_col,
                         label_col, num_epoch, communication_window, master_port, loss_weights, **kw)


class DOWNPOUR(AsynchronousDistributedTrainer):
    algorithm = "downpour"

    def __init__(self, keras_model, worker_optimizer, loss, metrics=None, num_workers=2, batch_size=32,
                 features_col="features", label_col="label", num_epoch=1, communication_window=5,
                 master_port=5000, loss_weights=None, **kw):
        super().__init__(keras_model, worker_optimizer, loss, metrics, num_workers, batch_size, features_col,
                         label_col, num_epoch, communication_window, master_port, loss_weights, **kw)


class EASGD(AsynchronousDistributedTrainer):
    """Elastic averaging SGD (synchronous rounds every ``communication_window`` batches)."""

    algorithm = "easgd"

    def __init__(self, keras_model, worker_optimizer, loss, metrics=None, features_col="features",
                 label_col="label", num_epoch=1, batch_size=32, num_workers=2, rho=5.0, learning_rate=0.1,
                 master_port=5000, loss_weights=None, communication_window=1, **kw):
        super().__init__(keras_model, worker_optimizer, loss, metrics, num_workers, batch_size, features_col,
                         label_col, num_epoch, communication_window, master_port, loss_weights,
                         alpha=min(1.0, float(rho) * float(learning_rate) / max(num_workers, 1)), **kw)
        self.rho, self.learning_rate = rho, learning_rate


class AEASGD(EASGD):
    algorithm = "aeasgd"

    def __init__(self, keras_model, worker_optimizer, loss, metrics=None, num_workers=2, batch_size=32,
                 features_col="features", label_col="label", num_epoch=1, communication_window=32, rho=5.0,
                 learning_rate=0.1, master_port=5000, loss_weights=None, **kw):
        super().__init__(keras_model, worker_optimizer, loss, metrics, features_col, label_col, num_epoch,
                         batch_size, num_workers, rho, learning_rate, master_port, loss_weights,
                         communication_window=communication_window, **kw)


class EAMSGD(EASGD):
    algorithm = "eamsgd"

    def __init__(self, keras_model, worker_optimizer, loss, metrics=None, num_workers=2, batch_size=32,
                 features_col="features", label_col="label", num_epoch=1, communication_window=32, rho=5.0,
                 learning_rate=0.1, momentum=0.9, master_port=5000, loss_weights=None, **kw):
        super().__init__(keras_model, worker_optimizer, loss, metrics, features_col, label_col, num_epoch,
                         batch_size, num_workers, rho, learning_rate, master_port, loss_weights,
                         communication_window=communication_window, momentum=momentum, **kw)


class SynchronousDataParallel(DistributedTrainer):
    """North-star trainer: per-step gradient all-reduce (RCCL, bucketed, overlapped)."""

    algorithm = "syncdp"

    def __init__(self, keras_model, worker_optimizer, loss, metrics=None, num_workers=2, batch_size=32,
                 features_col="features", label_col="label", num_epoch=1, bucket_mb=None, **kw):
        super().__init__(keras_model, worker_optimizer, loss, metrics, num_workers, batch_size, features_col,
                         label_col, num_epoch, 1, bucket_mb=bucket_mb, **kw)


SyncDP = SynchronousDataParallel

__all__ = ["Trainer", "SingleTrainer", "AveragingTrainer", "EnsembleTrainer", "DistributedTrainer",
           "AsynchronousDistributedTrainer", "ADAG", "DynSGD", "DOWNPOUR", "EASGD", "AEASGD", "EAMSGD",
           "SynchronousDataParallel", "SyncDP", "ParameterServer"]
