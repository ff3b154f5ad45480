"""Replica-batched execution of co-located recurrent workers: the R replicas of a ``ReplicaGroup``
(``parallel/replicas.py``) step as ONE launch per phase instead of R graph replays on R streams.

The reference's NYISO workload (``ddl_nyiso_aztk.py:195-218``; ``ddl_nyiso_hdi.ipynb:577-609``) trains
GRU(128) -> Dense(1) and LSTM(128) -> Dense(1) regressors with an MSE loss on ADAG workers, two per
executor.  Co-located on one MI355X, each replica step is a few latency-bound kernels on 32 batch
rows; run replica by replica, the GPU is mostly idle between them.  Here one step of ALL replicas is
(``csrc/kernels/rnn.hip``, ``rnn_replica_step``):

  1. the recurrent forward over R x B batch rows, each workgroup reading its replica's U / W / bias
     and its mini-batch from the replica's resident shard (index = device step counter % batches);
  2. the Dense head, MSE loss and their backward, one workgroup per replica (loss -> the replica's
     device history, Adam step tick);
  3. the recurrent backward over R x B rows;
  4. the recurrent parameter gradients, one grid slice per replica, written (not accumulated);
  5. one optimizer sweep over the R flat arenas, which also advances the step counter.

A commit window of ``k`` steps for all replicas is captured into ONE hipGraph and replayed per round;
the commit itself is the group's ``commit_replicas`` kernel, unchanged.

Ragged shards: the reference's ``repartition(num_workers)`` shards differ by a row
(``ddl_nyiso_aztk.py:193``; its 11,519 training rows give 2,880 / 2,880 / 2,880 / 2,879), so replicas take
different step counts.  Every replica fetches its own mini-batch (``ctr % nb_r``) and stays live while the
shared step counter is below its own step count; a replica past it is masked in the kernels (no history
slot, no Adam tick, no parameter or state update), which is exactly the per-replica schedule: an
exhausted worker stops stepping while the others finish their windows.  The update law, histories,
``num_updates`` and optimizer state are those of the per-replica path (tests/test_gpu_colocated.py
compares the two to fp32 rounding).
"""
from __future__ import annotations

import os

import torch

from ..models.step import graph_capture

from ..models import optimizers as opt_mod


def _layers(model):
    from ..models.core import Sequential
    from ..models.layers import GRU, LSTM, Dense

    if not isinstance(model, Sequential) or len(model.layers) != 2:
        return None
    rnn, dense = model.layers
    if type(rnn) not in (GRU, LSTM) or type(dense) is not Dense:
        return None
    return rnn, dense


MAX_R = 16  # kMaxRnnRep (csrc/include/ddl_ops.h): 8 executors x 2 processes


def why_not(group) -> str | None:
    """None when the group's replicas are RNN(64|128) -> Dense(K) / MSE fp32 models with a supported worker
    optimizer and at most 16 replicas (shards may be ragged); else the reason they are not batched."""
    if os.environ.get("DDL_REPLICA_BATCH", "1") == "0":
        return "DDL_REPLICA_BATCH=0"
    if not group.gpu or group.rule == "averaging":
        return "CPU group or averaging rule"
    reps = group.reps
    if not (1 < len(reps) <= MAX_R):
        return f"{len(reps)} replicas (batched: 2..{MAX_R})"
    from ..ops._native import C

    if len({r.bs for r in reps}) != 1:
        return "unequal batch sizes"
    for r in reps:
        m = r.model
        ls = _layers(m)
        if ls is None:
            return "not a GRU/LSTM -> Dense Sequential"
        if m.loss != "mean_squared_error" or m.arena.compute is not m.arena.master:
            return "loss is not MSE or compute is not fp32"
        rnn, dense = ls
        if (rnn.return_sequences or not rnn.use_bias or rnn.activation != "tanh"
                or rnn.recurrent_activation != "hard_sigmoid" or not rnn.trainable or not dense.trainable):
            return "recurrent layer outside the fused cell (return_sequences / no bias / activations / frozen)"
        if dense.activation_name not in (None, "linear") or dense.kernel.data.shape[1] != rnn.units:
            return "Dense head is not linear on the last hidden state"
        o = m.optimizer
        if getattr(o, "clipnorm", None) is not None or m.arena.numel % 4:
            return "clipnorm or arena size not a multiple of 4"
        if isinstance(o, opt_mod.SGD):
            if o.nesterov or o.dampening:
                return "SGD with nesterov / dampening"
        elif not isinstance(o, (opt_mod.Adagrad, opt_mod.Adam)):
            return f"worker optimizer {type(o).__name__}"
        X = r.X
        if X.dim() != 3 or X.dtype != torch.float32 or r.Y.dtype != torch.float32:
            return "inputs are not fp32 [rows, T, I]"
        if r.Y.numel() != r.Y.shape[0] * dense.units or not (X.is_contiguous() and r.Y.is_contiguous()):
            return "targets do not match the Dense head"
        if not C().rnn_replica_ok(rnn.cell, rnn.units, int(X.shape[2]), dense.units, r.bs):
            return f"H={rnn.units} / I={int(X.shape[2])} / K={dense.units} / batch={r.bs} outside the fused kernels"
    return None


def applies(group) -> bool:
    return why_not(group) is None


class BatchedReplicas:
    """Device state of the batched step for the replicas of one group (see module doc)."""

    def __init__(self, group):
        self.group = group
        reps = group.reps
        r0 = reps[0]
        rnn0, dense0 = _layers(r0.model)
        self.cell, self.H, self.K = rnn0.cell, rnn0.units, dense0.units
        self.T, self.I = int(r0.X.shape[1]), int(r0.X.shape[2])
        self.B, self.R = r0.bs, len(reps)
        self.nbs = [r.nb for r in reps]
        self.steps = [r.steps for r in reps]
        dev = r0.model.device
        G = 3 if self.cell == "gru" else 4
        RB, T, H = self.R * self.B, self.T, self.H
        f32 = dict(dtype=torch.float32, device=dev)
        self.hs = torch.empty((RB, T + 1, H), **f32)
        self.cs = torch.empty((RB, T + 1, H) if self.cell == "lstm" else (1,), **f32)
        self.gates = torch.empty((RB, T, G * H), **f32)
        self.hlast = torch.empty((RB, H), **f32)
        self.dh = torch.empty((RB, H), **f32)
        self.dgates = torch.empty((RB, T, G * H), **f32)
        self.ctr = torch.zeros(1, dtype=torch.int32, device=dev)
        self.live = torch.ones(self.R, dtype=torch.int32, device=dev)
        self.graph = None
        o = r0.model.optimizer
        if isinstance(o, opt_mod.Adam):
            self.opt, self.p1, self.p2 = 2, o.b1, o.b2
            self.amode = (1 if o.decoupled else 0) | (2 if o.keras_eps else 0)
        elif isinstance(o, opt_mod.Adagrad):
            self.opt, self.p1, self.p2, self.amode = 1, 0.0, 0.0, 0
        else:
            self.opt, self.p1, self.p2, self.amode = 0, o.momentum, 0.0, 0
        self.lr, self.eps, self.wd = o.lr, getattr(o, "eps", 0.0), o.weight_decay
        lists = {k: [] for k in ("xs", "ys", "Ws", "Us", "bs", "Wds", "bds", "gWs", "gUs", "gbs", "gWds", "gbds",
                                 "hists", "ws", "gs", "s1s", "s2s", "ts")}
        for r in reps:
            m = r.model
            rnn, dense = _layers(m)
            if self.opt == 2:
                m.optimizer.enable_device_step()
            lists["xs"].append(r.X)
            lists["ys"].append(r.Y.reshape(r.Y.shape[0], -1))
            lists["Ws"].append(rnn.kernel.data)
            lists["Us"].append(rnn.recurrent_kernel.data)
            lists["bs"].append(rnn.bias.data)
            lists["Wds"].append(dense.kernel.data)
            lists["bds"].append(None if dense.bias is None else dense.bias.data)
            lists["gWs"].append(rnn.kernel.grad)
            lists["gUs"].append(rnn.recurrent_kernel.grad)
            lists["gbs"].append(rnn.bias.grad)
            lists["gWds"].append(dense.kernel.grad)
            lists["gbds"].append(None if dense.bias is None else dense.bias.grad)
            lists["hists"].append(r.hist)
            lists["ws"].append(m.arena.master.detach())
            lists["gs"].append(m.arena.grad)
            st = m.optimizer.state
            lists["s1s"].append(st.get("m", st.get("acc", st.get("momentum"))))
            lists["s2s"].append(st.get("v"))
            lists["ts"].append(m.optimizer.device_step if self.opt == 2 else None)
        self.args = lists

    def _step(self):
        from ..ops._native import C

        a = self.args
        C().rnn_replica_step(self.cell, a["xs"], a["ys"], a["Ws"], a["Us"], a["bs"], a["Wds"], a["bds"], a["gWs"],
                             a["gUs"], a["gbs"], a["gWds"], a["gbds"], a["hists"], self.ctr, self.nbs, self.steps,
                             self.live, self.B,
                             self.hs, self.cs, self.gates, self.hlast, self.dh, self.dgates, a["ws"], a["gs"],
                             a["s1s"], a["s2s"], a["ts"], self.opt, self.lr, self.p1, self.p2, self.eps, self.wd,
                             self.amode)

    def run_steps(self, n: int):
        """n steps of every replica (eager launches on the current stream)."""
        for _ in range(n):
            self._step()
        self._advance(n)

    def capture(self, k: int) -> bool:
        """Capture a k-step window of all replicas into one hipGraph (False: capture failed, stay eager)."""
        dev = self.group.pg.device
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        g = torch.cuda.CUDAGraph()
        try:
            if os.environ.get("DDL_TEST_FAIL_CAPTURE") == "1":  # test hook: force the eager fallback
                raise RuntimeError("capture forced to fail (DDL_TEST_FAIL_CAPTURE)")
            with torch.cuda.stream(s):
                with graph_capture(g, s):
                    for _ in range(k):
                        self._step()
        except Exception as e:
            if os.environ.get("DDL_GRAPHS_STRICT") == "1":
                raise
            print(f"[ddl] batched replica hipGraph capture disabled: {type(e).__name__}: {e}", flush=True)
            torch.cuda.synchronize(dev)
            return False
        torch.cuda.current_stream(dev).wait_stream(s)
        self.graph, self.k = g, k
        return True

    def replay(self):
        self.graph.replay()
        self._advance(self.k)

    def _advance(self, n: int):
        for r in self.group.reps:  # host mirrors of the device counters (a replica stops at its own step count)
            took = max(0, min(n, r.steps - r.done))
            r.done += took
            r.model.optimizer.iterations += took
