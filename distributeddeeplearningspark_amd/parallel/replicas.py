"""In-process replica groups: the dist-keras workers that share one MI355X run as R model replicas
of ONE process, not as R processes time-slicing the GPU.

The reference runs ``num_processes`` replicas per executor (``spark.executor.cores = 2``,
``ddl_mnist_aztk.py:49-53,66``; ``ddl_nyiso_aztk.py:51-55``), each committing a window-normalised
delta to the parameter server every ``communication_window`` mini-batches
(``ddl_mnist_aztk.py:216-219``).  On one GPU those replicas are tiny (batch 16 / 32, 50K-1M
parameters): as separate OS processes each commit round cost a device synchronize plus a host
barrier, and most of the run was spent waiting for the slowest co-located peer.  Here:

  * one process per GPU holds its R replicas (own model, own flat arena, own worker-local
    optimizer state, own resident shard), plus the center variable;
  * every replica step is graph-replayed: a device-side step counter drives a ``batch_fetch``
    kernel that copies mini-batch ``index % batches_per_epoch`` of the resident shard into the
    graph's static inputs, and ``step_record`` appends the loss to a device history — so a whole
    window (``communication_window`` steps) of one replica is ONE hipGraph replay;
  * the R windows of a round run on R HIP streams (the replicas' kernels fill different CUs at the
    same time); the commit round is ONE kernel (``commit_replicas``) over the R arenas, ordered after
    the windows by stream events — no device synchronize, no host barrier;
  * with replicas on several GPUs (one process each) the kernel writes each GPU's partial sum of
    the deltas, which is all-reduced over RCCL before the apply.

The update law and ``num_updates`` are the multi-process ones (``trainers._CommitWorker``): in
round j the replicas with j < commits_r train ``k`` steps and commit ``s_r (W_r - c)``; exhausted
replicas run their leftover (< k) steps before their first non-contributing round and then commit
zero; the center sums the deltas in replica order, as the IPC exchange does, so the two paths agree
to fp32 rounding.  On the CPU the same schedule runs eagerly (tests compare it with the gloo
multi-process trainers).
"""
from __future__ import annotations

import os
import time

import torch

from ..models.step import graph_capture

COMMIT_RULES = ("adag", "dynsgd", "downpour", "easgd", "aeasgd", "eamsgd")
ELASTIC = ("easgd", "aeasgd", "eamsgd")


def mode() -> str:
    """``DDL_REPLICA_GROUPS``: ``auto`` (default: replicas co-located on a GPU run in one process),
    ``1`` (also on the CPU: one process for all workers), ``0`` (one OS process per worker), or an integer
    G > 1 (CPU tests of the multi-group path: the workers are dealt round-robin to G processes, as they are
    to the GPUs of a node)."""
    return os.environ.get("DDL_REPLICA_GROUPS", "auto")


def applies(cfg, devices) -> bool:
    if cfg.get("mode", "sync") != "sync" or cfg["algorithm"] not in COMMIT_RULES + ("averaging",):
        return False
    m = mode()
    if m == "0" or len(devices) < 2:
        return False
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:  # torchrun SPMD: k workers per rank, grouped by rank
        return len(set(devices)) < len(devices)
    if m == "1" or (m.isdigit() and int(m) > 1):
        return True
    return devices[0] != "cpu" and len(set(devices)) < len(devices)


def plan(devices) -> list[list[int]]:
    """Replica ids per group, one group per distinct device, in device order (CPU workers with
    ``DDL_REPLICA_GROUPS=G``: G round-robin groups)."""
    m = mode()
    if devices and devices[0] == "cpu" and m.isdigit() and int(m) > 1:
        g = min(int(m), len(devices))
        return [[r for r in range(len(devices)) if r % g == k] for k in range(g)]
    order: list[str] = []
    for d in devices:
        if d not in order:
            order.append(d)
    return [[r for r, d in enumerate(devices) if d == dev] for dev in order]


def _scale(rule, cfg, k, contrib, rid):
    if rid not in contrib:
        return 0.0
    if rule in ELASTIC:
        return float(cfg["alpha"])
    if rule == "adag":
        return 1.0 / k
    if rule == "dynsgd":
        return 1.0 / (contrib.index(rid) + 1)
    return 1.0


class _Replica:
    """One dist-keras worker: its model, resident shard and (GPU) graph-replayed step."""

    def __init__(self, rid, model, X, Y, steps, commits, bs):
        self.rid, self.model, self.bs = rid, model, bs
        self.X, self.Y = X, Y
        self.nb = max(1, X.shape[0] // bs)
        self.steps, self.commits = steps, commits
        self.done = 0  # steps taken (host mirror of the device counter)
        self.host_hist: list[float] = []
        dev = model.device
        self.gpu = dev.type == "cuda"
        if self.gpu:
            self.sx = torch.empty((bs,) + tuple(X.shape[1:]), dtype=X.dtype, device=dev)
            self.sy = torch.empty((bs,) + tuple(Y.shape[1:]), dtype=Y.dtype, device=dev)
            self.ctr = torch.zeros(1, dtype=torch.int32, device=dev)
            self.hist = torch.zeros(max(1, steps), dtype=torch.float32, device=dev)
            self.stream = torch.cuda.Stream(dev)
        self.graph = None

    # one step: fetch batch (ctr % nb) -> loss / backward -> optimizer -> record loss, ctr += 1
    def _step_body(self, captured: bool, more: bool = False):
        from ..ops._native import C
        from ..ops.scope import replica_scope

        m = self.model
        with replica_scope(self.rid):
            C().batch_fetch([self.X, self.Y], [self.sx, self.sy], self.ctr, self.nb)
            loss = m.backward_step(m.to_input(self.sx), m.to_target(self.sy))
            if captured:  # ``more``: another captured step follows (it skips its zero_grad fill)
                m.optimizer.captured_update(1.0, zero_grads=more)
                from ..models.step import _uses_dropout

                if _uses_dropout(m):  # fresh dropout masks on every replayed step (ops/act.py)
                    from ..ops.act import tick_dropout_step

                    tick_dropout_step(m.device)
            else:
                m.optimizer.step(1.0)
            C().step_record(loss.detach().float().reshape(1), self.hist, self.ctr)

    def run_steps(self, n: int):
        """``n`` steps on the current stream (GPU: eager launches; CPU: eager torch)."""
        if n <= 0:
            return
        m = self.model
        if not self.gpu:
            for _ in range(n):
                b = self.done % self.nb
                xb = self.X[b * self.bs:(b + 1) * self.bs]
                yb = self.Y[b * self.bs:(b + 1) * self.bs]
                loss = m.backward_step(m.to_input(xb), m.to_target(yb))
                m.optimizer.step(1.0)
                self.host_hist.append(float(loss.detach()))
                self.done += 1
            return
        for _ in range(n):
            self._step_body(captured=False)
            self.done += 1

    def capture_window(self, k: int, stream):
        """Capture k steps into one graph (the device step counters advance on every replay)."""
        m = self.model
        m.optimizer.enable_device_step()
        g = torch.cuda.CUDAGraph()
        with graph_capture(g, stream):
            for i in range(k):
                self._step_body(captured=True, more=i + 1 < k)
        from ..ops.norm import _POOL

        # the replayed kernels address the statistics-pool buffers: keep them alive even if the
        # (global) pool is regrown later by another model (as models/step.py does)
        self._keep = list(_POOL.buf.values())
        self.graph = g
        self.k = k

    def replay_window(self):
        self.graph.replay()
        self.done += self.k
        self.model.optimizer.iterations += self.k  # host mirror of the device step counter

    def losses(self) -> list[float]:
        if self.gpu:
            return self.hist[: min(self.done, self.hist.numel())].tolist()
        return self.host_hist


class ReplicaGroup:
    """The R replicas of one device and their commit rounds (see module doc)."""

    def __init__(self, cfg, blob, Xs, Ys, rids, sizes, pg):
        from ..models import optimizers as opt_mod
        from ..utils import deserialize_keras_model, set_states

        self.cfg, self.pg, self.rids = cfg, pg, list(rids)
        self.rule = cfg["algorithm"]
        bs, E = int(cfg["batch_size"]), int(cfg["num_epoch"])
        self.k = max(1, int(cfg.get("communication_window", 1)))
        self.steps_all = [E * (s // bs) for s in sizes]
        self.commits_all = [st // self.k for st in self.steps_all]
        self.rounds = max(self.commits_all) if self.commits_all else 0
        dev = pg.device
        self.gpu = dev.type == "cuda"
        self.reps: list[_Replica] = []
        for rid, X, Y in zip(rids, Xs, Ys):
            model = deserialize_keras_model({k: v for k, v in blob.items() if k not in ("optimizer", "loss")})
            opt = opt_mod.get(cfg["worker_optimizer"])
            if self.rule == "eamsgd" and isinstance(opt, opt_mod.SGD) and not opt.momentum:
                opt.momentum = cfg.get("momentum", 0.9)
            model.compile(opt, cfg["loss"])
            model.seed = cfg.get("seed", 0)
            model.place(dev)
            if blob.get("flat") is not None:
                model.arena.set_flat(torch.from_numpy(blob["flat"]))
            if blob.get("states"):
                set_states(model, blob["states"])
            Xd, Yd = self._resident(X, model), self._resident(Y, model, labels=True)
            self.reps.append(_Replica(rid, model, Xd, Yd, self.steps_all[rid], self.commits_all[rid], bs))
        a0 = self.reps[0].model.arena
        self.center = a0.master.detach().clone()
        self.sum = torch.zeros_like(self.center) if (pg.distributed and self.gpu) else None
        self.commit_s = 0.0
        self.graph_rounds = 0
        self.batched = None  # replica_batch.BatchedReplicas when the replicas step as one launch per phase
        self.batch_reason = None  # why a GPU group runs per-replica instead (logged once, in the results)

    @staticmethod
    def _resident(a, model, labels=False):
        t = torch.from_numpy(a) if not isinstance(a, torch.Tensor) else a
        t = t.to(model.device)
        if not labels and t.is_floating_point() and t.dtype != model.compute_dtype:
            t = t.to(model.compute_dtype)  # once, not per batch
        return t.contiguous()

    def num_updates(self) -> int:
        if self.rule == "averaging":
            return 1
        return int(sum(self.commits_all))

    # ---------------------------------------------------------------- commit round
    def _commit(self, j: int):
        t0 = time.perf_counter()
        contrib = [r for r, c in enumerate(self.commits_all) if j < c]
        scales = [_scale(self.rule, self.cfg, self.k, contrib, rep.rid) for rep in self.reps]
        elastic = self.rule in ELASTIC
        if self.gpu:
            from ..ops._native import C

            ws = [r.model.arena.master.detach() for r in self.reps]
            w16 = [None if r.model.arena.compute is r.model.arena.master else r.model.arena.compute for r in self.reps]
            if self.sum is None:
                C().commit_replicas(ws, w16, scales, self.center, None, elastic, 0)
            else:
                from .ddp import all_reduce_flat

                C().commit_replicas(ws, w16, scales, self.center, self.sum, elastic, 1)
                all_reduce_flat(self.pg, self.sum, 64 << 20)
                C().commit_replicas(ws, w16, scales, self.center, self.sum, elastic, 2)
        else:
            self._commit_host(scales, elastic)
        self.commit_s += time.perf_counter() - t0

    def _commit_host(self, scales, elastic):
        c0 = self.center
        with torch.no_grad():
            acc = torch.zeros_like(c0) if self.pg.distributed else c0.clone()
            for rep, s in zip(self.reps, scales):
                W = rep.model.arena.master.detach()
                x = (W - c0) * s
                acc.add_(x)
                if elastic:
                    W.sub_(x)
            if self.pg.distributed:
                from .ddp import all_reduce_flat

                all_reduce_flat(self.pg, acc, 64 << 20)
                acc.add_(c0)
            c0.copy_(acc)
            for rep in self.reps:
                if not elastic:
                    rep.model.arena.master.detach().copy_(c0)
                rep.model.arena.sync_compute()

    # ---------------------------------------------------------------- schedule
    def _window_all(self, todo: list[_Replica], n: int, use_graphs: bool):
        """n steps of each replica in ``todo``: concurrent streams on the GPU."""
        if not todo:
            return
        if not self.gpu:
            for rep in todo:
                rep.run_steps(n)
            return
        main = torch.cuda.current_stream(self.pg.device)
        for rep in todo:
            rep.stream.wait_stream(main)
            with torch.cuda.stream(rep.stream):
                if use_graphs and rep.graph is not None and n == self.k:
                    rep.replay_window()
                else:
                    rep.run_steps(n)
        for rep in todo:
            main.wait_stream(rep.stream)

    def run(self):
        from ..models.step import graphs_enabled

        k = self.k
        graphs = self.gpu and graphs_enabled() and all(getattr(r.model, "graph_capturable", True) and
                                                        getattr(r.model.optimizer, "clipnorm", None) is None
                                                        for r in self.reps)
        warm_rounds = max(1, -(-2 // k))  # eager rounds first: workspaces settle (2 eager steps, as step.py)
        if self.rule == "averaging":
            for rep in self.reps:
                self._window_all([rep], rep.steps, False)
            self._average()
            return
        if self._try_batched():
            self._run_batched(graphs)
            return
        for j in range(self.rounds):
            todo = [r for r in self.reps if j < r.commits]
            if graphs and j == warm_rounds:
                graphs = self._capture(todo)
            self._window_all(todo, k, graphs and j >= warm_rounds)
            # exhausted replicas: their leftover (< k) steps come before their first zero commit
            for r in self.reps:
                if j == r.commits and r.steps > r.done:
                    self._window_all([r], r.steps - r.done, False)
            self._commit(j)
        for r in self.reps:  # steps after the last commit round (history only)
            if r.steps > r.done:
                self._window_all([r], r.steps - r.done, False)
        if self.gpu:
            torch.cuda.synchronize(self.pg.device)

    def _try_batched(self) -> bool:
        """Pick the one-launch-per-op path for this group's replicas when one applies: recurrent regressors
        (NYISO, ``replica_batch``) or Sequential CNN / MLP classifiers (MNIST, ``replica_seq``).  When neither
        does, log one line with the reason (the per-replica path is several times slower on these tiny
        models) and keep it in ``self.batch_reason`` for the result dicts."""
        from . import replica_batch, replica_seq

        if not self.gpu:
            return False
        why_rnn = replica_batch.why_not(self)
        if why_rnn is None:
            self.batched = replica_batch.BatchedReplicas(self)
            return True
        why_seq = replica_seq.why_not(self)
        if why_seq is None:
            try:
                self.batched = replica_seq.SeqReplicas(self)
                return True
            except ValueError as e:  # a launch-plan shape the batched kernels do not cover: per-replica path
                why_seq = str(e)
        is_rnn = replica_batch._layers(self.reps[0].model) is not None
        self.batch_reason = why_rnn if is_rnn else why_seq
        if self.batch_reason != "DDL_REPLICA_BATCH=0":
            print(f"[ddl] replica group of {len(self.reps)} runs per replica (not batched): {self.batch_reason}",
                  flush=True)
        return False

    def _run_batched(self, graphs: bool):
        """Every replica steps in lockstep on one device step counter: round j = one k-step window of ALL
        replicas (one hipGraph replay from round 1 on; round 0 runs eagerly) + the commit kernel.  Ragged
        shards: a replica whose steps run out is masked on the device (it stops, the others finish their
        windows), as in the per-replica schedule."""
        bat, k = self.batched, self.k
        for j in range(self.rounds):
            if graphs and j == 1 and bat.graph is None:
                graphs = bat.capture(k)
            if graphs and bat.graph is not None:
                bat.replay()
                self.graph_rounds += 1
            else:
                bat.run_steps(k)
            self._commit(j)
        left = max(r.steps - r.done for r in self.reps)  # steps after the last commit round (history only)
        if left > 0:
            bat.run_steps(left)
        torch.cuda.synchronize(self.pg.device)

    def _capture(self, reps) -> bool:
        """Capture every replica's window; on failure fall back to eager windows (capture is an
        optimisation, as in ``models/step.py``) and return False."""
        main = torch.cuda.current_stream(self.pg.device)
        torch.cuda.synchronize(self.pg.device)
        try:
            if os.environ.get("DDL_TEST_FAIL_CAPTURE") == "1":  # test hook: force the fallback path
                raise RuntimeError("capture forced to fail (DDL_TEST_FAIL_CAPTURE)")
            for rep in reps:
                rep.stream.wait_stream(main)
                rep.capture_window(self.k, rep.stream)
        except Exception as e:
            if os.environ.get("DDL_GRAPHS_STRICT") == "1":
                raise
            print(f"[ddl] replica-group hipGraph capture disabled: {type(e).__name__}: {e}", flush=True)
            for rep in self.reps:
                rep.graph = None
                rep.model.arena.grads_zeroed = False  # a capture cut short must not skip an eager fill
            torch.cuda.synchronize(self.pg.device)
            return False
        for rep in reps:
            main.wait_stream(rep.stream)
        return True

    def _average(self):
        """AveragingTrainer: independent training, then the mean of all replicas' weights."""
        with torch.no_grad():
            acc = torch.zeros_like(self.center)
            for rep in self.reps:
                acc.add_(rep.model.arena.master.detach())
            if self.pg.distributed:
                from .ddp import all_reduce_flat

                all_reduce_flat(self.pg, acc, 64 << 20)
            acc.div_(len(self.steps_all))
            self.center.copy_(acc)
            for rep in self.reps:
                rep.model.arena.master.detach().copy_(acc)
                rep.model.arena.sync_compute()


def train_group(rank, world, pg, cfg, blob, Xs, Ys, rids, sizes):
    """Executor entry point: train this device's replicas; one result dict per replica."""
    from ..utils import get_states

    t0 = time.time()
    grp = ReplicaGroup(cfg, blob, Xs, Ys, rids, sizes, pg)
    grp.run()
    elapsed = time.time() - t0
    out = []
    for i, rep in enumerate(grp.reps):
        res = {"rank": rep.rid, "history": rep.losses(), "num_updates": grp.num_updates(), "time": elapsed,
               "commit_s": grp.commit_s, "commit_wait_s": None, "commit_xfer_s": None,
               "graph": (grp.batched.graph is not None) if grp.batched is not None else rep.graph is not None,
               "ingest": "resident", "timed_s": None, "timed_steps": 0,
               "replica_group": {"group": rank, "groups": world, "replicas": len(grp.reps),
                                 "batched": grp.batched is not None, "batch_reason": grp.batch_reason}}
        if rep.rid == 0:
            res["flat"] = grp.reps[0].model.arena.to_canonical(grp.center).cpu().numpy().copy()
            res["states"] = get_states(rep.model)
        out.append(res)
    return out
