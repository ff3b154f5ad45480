"""Replica-batched execution of co-located Keras ``Sequential`` CNN / MLP workers: the R replicas of a
``ReplicaGroup`` (``parallel/replicas.py``) step as ONE launch per op instead of R graph replays.

The reference's MNIST workflow (``ddl_mnist_aztk.py:180-199,212-219``) trains a Conv2D(32) -> Conv2D(32)
-> MaxPool -> Dense(225) -> Dense(10) softmax network with Adam on batches of 16, two workers per
executor (``ddl_mnist_aztk.py:49-53,66``).  Co-located on one MI355X, one replica step is ~25 small
kernels (each a few workgroups); stepping R replicas on R streams keeps the GPU mostly idle between
them.  Here the replicas' parameter arenas are stacked in one [R, numel] allocation (``ParamArena.rebind``),
so every op addresses replica z's weights at a fixed stride and runs as ONE launch over all R mini-batches:

  * the GEMMs / implicit-GEMM convolutions take a replica grid dimension (``GemmParams::zcount``:
    operands, output and bias at z * stride);
  * the bias gradients (with the ReLU backward fused), the split-K finalize (per-replica bias), the
    flipped dgrad filters and the softmax-xent loss (one loss per replica) take the same dimension;
  * pooling / padding work on the stacked batch as is;
  * ONE optimizer launch sweeps the stacked arenas (shared device step counter: the replicas step in
    lockstep), zeroing the gradients as it goes; one ``batch_fetch`` / ``step_record`` serve all replicas.

A commit window of ``k`` steps for all replicas is one hipGraph, replayed per round; the commit is the
group's ``commit_replicas`` kernel, unchanged.

Ragged shards (``repartition(num_workers)`` of 59,999 rows gives shards a row apart,
``ddl_mnist_aztk.py:156``) and up to 16 replicas (8 executors x 2 processes, ``ddl_mnist_aztk.py:49-53``):
each replica fetches mini-batch ``ctr % nb_r`` of its own shard, and the stacked optimizer
(``replica.hip`` ``opt_stack_step``) and ``step_record`` mask a replica once the shared step counter
reaches its own step count, so an exhausted worker stops while the others finish their windows (the
per-replica schedule).  Each replica keeps its own Adam step counter.  Update law, histories, ``num_updates`` and optimizer state are
those of the per-replica path (tests/test_gpu_colocated.py compares the two).
"""
from __future__ import annotations

import math
import os

import torch

from ..models.step import graph_capture

from ..models import optimizers as opt_mod

_MAX_R = 16  # kMaxBatchCopies / 2 (csrc/include/ddl_ops.h)


def _plan(model):
    """[(kind, layer, relu)] for a supported Sequential (conv / pool / flatten / dense ..., softmax head), or None."""
    from ..models.core import Sequential
    from ..models.layers import Activation, Conv2D, Dense, Flatten, MaxPooling2D

    if not isinstance(model, Sequential):
        return None
    L, ops, i = model.layers, [], 0
    flat = len(tuple(model.input_shape)) == 1  # a Dense reads [rows, features]: 1-D input or after a Flatten
    while i < len(L):
        l = L[i]
        nxt = L[i + 1] if i + 1 < len(L) else None
        relu_next = isinstance(nxt, Activation) and nxt.activation_name == "relu"
        if isinstance(l, Conv2D):
            if l.strides != (1, 1) or l.dilation_rate != (1, 1) or not l.trainable:
                return None
            if l.activation_name not in ("linear", "relu") or l.filters % 8 or flat:
                return None
            ops.append(("conv", l, l.activation_name == "relu" or relu_next))
        elif isinstance(l, MaxPooling2D):
            if l.padding != "valid" or l.pool_size != l.strides or flat:
                return None
            ops.append(("pool", l, False))
        elif isinstance(l, Flatten):
            ops.append(("flatten", l, False))
            flat = True
        elif isinstance(l, Dense):
            if not l.trainable or not flat:  # a Dense on a 4-D activation is not a [rows, K] GEMM here
                return None
            last = i == len(L) - 1 or (i == len(L) - 2 and isinstance(nxt, Activation) and nxt.activation_name == "softmax")
            if last:
                if l.activation_name not in ("softmax", "linear") or (l.activation_name == "linear" and nxt is None):
                    return None
                ops.append(("head", l, False))
                return ops
            if l.activation_name not in ("linear", "relu"):
                return None
            ops.append(("dense", l, l.activation_name == "relu" or relu_next))
        elif isinstance(l, Activation):
            if l.activation_name != "relu" or not ops or ops[-1][0] not in ("conv", "dense"):
                return None  # a ReLU directly after conv / dense is fused into it
        else:
            return None
        i += 1
    return None


def why_not(group) -> str | None:
    """None when the group's replicas are co-located Sequential CNN / MLP classifiers with a softmax
    cross-entropy head, Adam / SGD(+momentum), bf16 compute and at most 16 replicas (shards may be ragged);
    else the reason they are not batched."""
    if os.environ.get("DDL_REPLICA_BATCH", "1") == "0":
        return "DDL_REPLICA_BATCH=0"
    if not group.gpu or group.rule == "averaging":
        return "CPU group or averaging rule"
    from ..ops import determinism as _det

    reps = group.reps
    if not (1 < len(reps) <= _MAX_R):
        return f"{len(reps)} replicas (batched: 2..{_MAX_R})"
    if _det.enabled():
        return "deterministic mode (the batched weight gradients split K with atomics)"
    if len({r.bs for r in reps}) != 1:
        return "unequal batch sizes"
    for r in reps:
        m = r.model
        if _plan(m) is None:
            return "layer stack outside the batched plan (conv / pool / flatten / dense with a softmax head)"
        if m.compute_dtype != torch.bfloat16 or not getattr(m, "graph_capturable", True):
            return "compute dtype is not bf16 or the model is not graph-capturable"
        if m.loss not in ("categorical_crossentropy", "sparse_categorical_crossentropy"):
            return f"loss {m.loss}"
        o = m.optimizer
        if getattr(o, "clipnorm", None) is not None or type(o) not in (opt_mod.Adam, opt_mod.AdamW, opt_mod.SGD):
            return f"worker optimizer {type(o).__name__} (or clipnorm)"
        if isinstance(o, opt_mod.SGD) and (o.nesterov or o.dampening):
            return "SGD with nesterov / dampening"
        if r.X.dtype != torch.bfloat16 or not r.X.is_contiguous() or not r.Y.is_contiguous():
            return "shard is not contiguous bf16"
        K = m.layers[-1].units if hasattr(m.layers[-1], "units") else m.layers[-2].units
        if r.bs * len(reps) > 4096 or r.bs * K * len(reps) > 65536 or len(reps) * r.bs > 1024:
            return "stacked batch too large for the one-launch loss"
        if m.loss == "categorical_crossentropy" and (r.Y.dtype != torch.float32 or r.Y.numel() != r.Y.shape[0] * K):
            return "one-hot targets are not fp32 [rows, K]"
        if m.loss == "sparse_categorical_crossentropy" and (r.Y.dtype != torch.int64 or r.Y.numel() != r.Y.shape[0]):
            return "sparse targets are not int64 [rows]"
    return None


def applies(group) -> bool:
    return why_not(group) is None


class SeqReplicas:
    """Device state and launch sequence of the batched step (see module doc)."""

    def __init__(self, group):
        from ..ops import conv as CV
        from ..ops import gemm as G

        self.group = group
        reps = group.reps
        self.R, self.B = len(reps), reps[0].bs
        self.nbs = [r.nb for r in reps]
        m0 = reps[0].model
        dev = m0.device
        self.dev = dev
        R, B = self.R, self.B
        self.ops = _plan(m0)
        self.sparse = m0.loss == "sparse_categorical_crossentropy"
        # ---- stacked arenas: replica z's parameters at z * NW elements
        a0 = m0.arena
        NW = self.NW = a0.numel
        self.W = torch.empty((R, NW), dtype=torch.float32, device=dev)
        self.Gr = torch.zeros((R, NW), dtype=torch.float32, device=dev)
        self.W16 = torch.empty((R, NW), dtype=torch.bfloat16, device=dev)
        for z, r in enumerate(reps):
            a = r.model.arena
            self.W[z].copy_(a.master.detach())
            self.W16[z].copy_(a.compute.detach())
            a.rebind(self.W[z], self.Gr[z], self.W16[z])
        # ---- optimizer: one launch over the stacked arenas; per-replica step counts (ragged shards)
        o0 = m0.optimizer
        self.adam = isinstance(o0, opt_mod.Adam)
        self.state = {}
        for k in o0.state:
            st = torch.zeros((R, NW), dtype=torch.float32, device=dev)
            for z, r in enumerate(reps):
                st[z].copy_(r.model.optimizer.state[k])
                r.model.optimizer.state[k] = st[z]
            self.state[k] = st
        self.ts = torch.tensor([float(r.model.optimizer.iterations) for r in reps], dtype=torch.float32, device=dev)
        self.steps_lim = torch.tensor([r.steps for r in reps], dtype=torch.int32, device=dev)
        self.opt = o0
        # ---- data: one fetch for all replicas into the stacked batch
        X0, Y0 = reps[0].X, reps[0].Y
        self.sx = torch.empty((R * B,) + tuple(X0.shape[1:]), dtype=X0.dtype, device=dev)
        self.sy = torch.empty((R * B,) + tuple(Y0.shape[1:]), dtype=Y0.dtype, device=dev)
        self.srcs = [r.X for r in reps] + [r.Y for r in reps]
        self.dsts = [self.sx[z * B:(z + 1) * B] for z in range(R)] + [self.sy[z * B:(z + 1) * B] for z in range(R)]
        self.ctr = torch.zeros(1, dtype=torch.int32, device=dev)
        cap = max(1, max(r.steps for r in reps))
        self.hist = torch.zeros((R, cap), dtype=torch.float32, device=dev)
        for z, r in enumerate(reps):
            r.hist = self.hist[z]
        self.loss = torch.zeros(R, dtype=torch.float32, device=dev)
        self.graph = None
        self._build(CV, G)

    # ------------------------------------------------------------------ static launch plan
    def _build(self, CV, G):
        """Shapes, buffers and per-op launch arguments (allocated once: graph-capturable)."""
        R, B, NW, dev = self.R, self.B, self.NW, self.dev
        bf = dict(dtype=torch.bfloat16, device=dev)
        shape = tuple(self.group.reps[0].model.input_shape)  # per-sample, storage width below
        width = shape[-1]
        x = self.sx
        steps = []
        for kind, l, relu in self.ops:
            st = {"kind": kind, "layer": l, "relu": relu}
            if kind == "conv":
                H, W_, Ci = shape
                kp, bp = l.kernel, l.bias
                Cop, KH, KW, Cip = kp.pshape
                if width != Cip:  # pad the input channels (the 1-channel MNIST image: 1 -> 8)
                    st["pad_in"] = (x, torch.empty((R * B, H, W_, Cip), **bf))
                    x = st["pad_in"][1]
                (ph, pw), extra = l._pads(H, W_)
                if extra is not None:
                    raise ValueError("replica_seq: asymmetric 'same' padding")
                g = CV.geometry(B, H, W_, Cip, Cop, KH, KW, (1, 1), (ph, pw), (1, 1))
                if not (g.implicit_fwd or g.gather8_fwd) or not (g.implicit_wgrad or g.gather8_wgrad):
                    raise ValueError("replica_seq: conv shape outside the gathered implicit GEMM")
                y = torch.empty((R * B, g.Ho, g.Wo, Cop), **bf)
                st.update(x=x, y=y, g=g, w=kp, b=bp, Cip=Cip, Cop=Cop,
                          tile=G.choose_tile(R * g.M, Cop))
                st["dy"] = torch.empty_like(y) if relu else None
                st["dx"] = torch.empty((R * B, H, W_, Cip), **bf)
                g2 = CV._dgrad_as_forward(g)
                st["g2"] = g2
                if g2 is not None:
                    st["wflip"] = torch.empty((R, Cip, KH, KW, Cop), **bf)
                # weight gradient: split K (pixels) so R x tiles x splits fills the chip twice
                bn_cap = min(128, Cip) if g.implicit_wgrad else 128
                wt = G.choose_tile(Cop, g.T * Cip, bn_cap)
                bm_, bn_ = G._TILES[wt]
                tiles = math.ceil(Cop / bm_) * math.ceil(g.T * Cip / bn_)
                splits = max(1, min(math.ceil(512 / (tiles * R)), g.M // 256))
                st["wg"] = (wt, math.ceil(g.M / splits / 64) * 64)
                x, shape, width = y, (g.Ho, g.Wo, l.filters), Cop
            elif kind == "pool":
                H, W_, Cc = shape
                kh, kw = l.pool_size
                Ho, Wo = (H - kh) // kh + 1, (W_ - kw) // kw + 1
                y = torch.empty((R * B, Ho, Wo, width), **bf)
                st.update(x=x, y=y, am=torch.empty((R * B, Ho, Wo, width), dtype=torch.uint8, device=dev),
                          dx=torch.empty_like(x))
                x, shape = y, (Ho, Wo, Cc)
            elif kind == "flatten":
                if width != shape[-1]:
                    raise ValueError("replica_seq: flatten of channel-padded activations")
                F_ = int(math.prod(shape))
                st.update(inshape=x.shape)
                x, shape, width = x.reshape(R * B, F_), (F_,), F_
            else:  # dense / head
                K = shape[-1]
                kp, bp = l.kernel, l.bias
                Np, Kp = kp.pshape
                if width != Kp:
                    st["pad_in"] = (x, torch.empty((R * B, Kp), **bf))
                    x = st["pad_in"][1]
                y = torch.empty((R * B, Np), **bf)
                tiles = math.ceil(B / 64) * math.ceil(Np / 64)
                skinny = Kp >= 1024 and tiles <= G._SKINNY_FWD_TILES and kind == "dense"
                st.update(x=x, y=y, w=kp, b=bp, K=K, Kp=Kp, Np=Np, N=l.units,
                          tile=G.choose_tile(R * B, Np), skinny=skinny,
                          wtile=G.choose_tile(Np, Kp), dx=torch.empty((R * B, Kp), **bf),
                          dy=torch.empty_like(y) if relu else None)
                if skinny:
                    splits = max(2, min(math.ceil(512 / (tiles * R)), Kp // 256))  # ~2 workgroups per CU
                    st["ks"] = math.ceil(Kp / splits / 64) * 64
                    st["ws"] = torch.zeros((R * B, Np), dtype=torch.float32, device=dev)
                x, shape, width = y, (l.units,), Np
            steps.append(st)
        head = steps[-1]
        head["dl"] = torch.empty_like(head["y"])
        self.steps = steps

    # parameter p of EVERY replica: the stacked buffer from replica 0's copy of p on (one base pointer + the
    # replica stride NW; the launch checks read the extent of all R copies from it)
    def _m(self, p):
        return self.W.view(-1)[p.offset:]

    def _g(self, p):
        return self.Gr.view(-1)[p.offset:]

    # ------------------------------------------------------------------ one step of every replica
    def _step(self):
        from ..ops import gemm as G
        from ..ops._native import C

        c = C()
        R, B, NW = self.R, self.B, self.NW
        c.batch_fetch(self.srcs, self.dsts, self.ctr, self.nbs + self.nbs)
        # ---------------- forward
        for st in self.steps:
            kind = st["kind"]
            if kind == "conv":
                if "pad_in" in st:
                    c.pad_cols_bf16(*st["pad_in"])
                g, Cip, Cop = st["g"], st["Cip"], st["Cop"]
                mode = G.KC_GATHER if g.implicit_fwd else G.KC_GATHER8
                b = st["b"]
                c.gemm(st["x"], st["w"].pdata, st["y"], g.M, Cop, g.T * Cip, mode, G.KC, 0, g.T * Cip, Cop, G.EPI_BF16,
                       st["tile"], max(64, math.ceil(g.T * Cip / 64) * 64), bias=None if b is None else self._m(b),
                       relu=int(st["relu"]), geom=g.fwd_geom, zcount=R, za=B * g.H * g.W * Cip, zb=NW,
                       zc=g.M * Cop, zbias=NW if b is not None else 0)
            elif kind == "pool":
                kh, kw = st["layer"].pool_size
                c.maxpool_fwd(st["x"], st["y"], st["am"], kh, kw, kh, kw, 0, 0)
            elif kind in ("dense", "head"):
                if "pad_in" in st:
                    c.pad_cols_bf16(*st["pad_in"])
                Kp, Np, b = st["Kp"], st["Np"], st["b"]
                bias = None if b is None else self._m(b)
                if st["skinny"]:
                    c.gemm(st["x"], st["w"].pdata, st["ws"], B, Np, Kp, G.KC, G.KC, Kp, Kp, Np, G.EPI_F32_ATOMIC, 3,
                           st["ks"], zcount=R, za=B * Kp, zb=NW, zc=B * Np)
                    c.splitk_finalize(st["ws"], st["y"], Np, bias, bool(st["relu"]), None, 0, brows=B, zbias=NW)
                else:
                    c.gemm(st["x"], st["w"].pdata, st["y"], B, Np, Kp, G.KC, G.KC, Kp, Kp, Np, G.EPI_BF16, st["tile"],
                           max(64, math.ceil(Kp / 64) * 64), bias=bias, relu=int(st["relu"]), zcount=R, za=B * Kp,
                           zb=NW, zc=B * Np, zbias=NW if b is not None else 0)
        # ---------------- loss: softmax cross-entropy, one loss per replica
        head = self.steps[-1]
        N, Np = head["N"], head["Np"]
        lg, dl = head["y"][:, :N], head["dl"][:, :N]
        if self.sparse:
            c.softmax_xent(lg, self.sy.reshape(-1), None, None, dl, 1.0 / B, 0.0, -100, None, self.loss, 1.0 / B, B)
        else:
            c.softmax_xent(lg, None, self.sy, None, dl, 1.0 / B, 0.0, -100, None, self.loss, 1.0 / B, B)
        # ---------------- backward
        d = head["dl"]
        for i in range(len(self.steps) - 1, -1, -1):
            st = self.steps[i]
            kind = st["kind"]
            first = i == 0
            if kind in ("dense", "head"):
                Kp, Np, b, w = st["Kp"], st["Np"], st["b"], st["w"]
                if st["relu"]:
                    if b is not None:
                        c.bias_grad(d, self._g(b), Np, True, st["y"], st["dy"], zcount=R, zdb=NW)
                    else:
                        c.relu_bwd(d, st["y"], st["dy"])
                    d = st["dy"]
                elif b is not None:
                    c.bias_grad(d, self._g(b), Np, True, zcount=R, zdb=NW)
                c.gemm(d, st["x"], self._g(w), Np, Kp, B, G.RC, G.RC, Np, Kp, Kp, G.EPI_F32, st["wtile"],
                       max(64, math.ceil(B / 64) * 64), zcount=R, za=B * Np, zb=B * Kp, zc=NW)
                if not first:
                    c.gemm(d, w.pdata, st["dx"], B, Kp, Np, G.KC, G.RC, Np, Kp, Kp, G.EPI_BF16, G.choose_tile(R * B, Kp),
                           max(64, math.ceil(Np / 64) * 64), zcount=R, za=B * Np, zb=NW, zc=B * Kp)
                    d = st["dx"]
            elif kind == "flatten":
                d = d.view(st["inshape"])
            elif kind == "pool":
                kh, kw = st["layer"].pool_size
                c.maxpool_bwd(d, st["am"], st["dx"], kh, kw, kh, kw, 0, 0)
                d = st["dx"]
            else:  # conv
                g, Cip, Cop, b, w = st["g"], st["Cip"], st["Cop"], st["b"], st["w"]
                if st["relu"]:
                    if b is not None:
                        c.bias_grad(d, self._g(b), Cop, True, st["y"], st["dy"], zcount=R, zdb=NW)
                    else:
                        c.relu_bwd(d, st["y"], st["dy"])
                    d = st["dy"]
                elif b is not None:
                    c.bias_grad(d, self._g(b), Cop, True, zcount=R, zdb=NW)
                wt, ks = st["wg"]
                bmode = G.RC_GATHER if g.implicit_wgrad else G.RC_GATHER8
                c.gemm(d, st["x"], self._g(w), Cop, g.T * Cip, g.M, G.RC, bmode, Cop, 0, g.T * Cip,
                       G.EPI_F32_ATOMIC if ks < g.M else G.EPI_F32, wt, ks, geom=g.fwd_geom, zcount=R, za=g.M * Cop,
                       zb=B * g.H * g.W * Cip, zc=NW)
                if not first:
                    g2 = st["g2"]
                    c.filter_taps_transpose(w.pdata, st["wflip"], list(range(g.T - 1, -1, -1)), zcount=R, zw=NW)
                    mode = G.KC_GATHER if g2.implicit_fwd else G.KC_GATHER8
                    c.gemm(d, st["wflip"], st["dx"], g2.M, g2.Co, g2.T * g2.Ci, mode, G.KC, 0, g2.T * g2.Ci, g2.Co,
                           G.EPI_BF16, G.choose_tile(R * g2.M, g2.Co),
                           max(64, math.ceil(g2.T * g2.Ci / 64) * 64), geom=g2.fwd_geom, zcount=R,
                           za=g.M * Cop, zb=g2.T * g2.Ci * g2.Co, zc=g2.M * g2.Co)
                    d = st["dx"]
        # ---------------- optimizer over the stacked arenas (live replicas only, + gradient zeroing)
        o = self.opt
        if self.adam:
            c.opt_stack_step(2, self.W, self.Gr, self.state["m"], self.state["v"], self.W16, self.ctr, self.steps_lim,
                             self.ts, o.lr, 0.0, o.b1, o.b2, o.eps, o.weight_decay,
                             (1 if o.decoupled else 0) | (2 if o.keras_eps else 0))
        else:
            mom = self.state.get("momentum") if o.momentum else None
            c.opt_stack_step(0, self.W, self.Gr, mom, None, self.W16, self.ctr, self.steps_lim, None, o.lr,
                             float(o.momentum), 0.0, 0.0, 0.0, o.weight_decay, 0)
        c.step_record(self.loss, self.hist, self.ctr, self.steps_lim, self.ts)

    # ------------------------------------------------------------------ schedule (BatchedReplicas interface)
    def run_steps(self, n: int):
        for _ in range(n):
            self._step()
        self._advance(n)

    def capture(self, k: int) -> bool:
        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        g = torch.cuda.CUDAGraph()
        try:
            if os.environ.get("DDL_TEST_FAIL_CAPTURE") == "1":
                raise RuntimeError("capture forced to fail (DDL_TEST_FAIL_CAPTURE)")
            with torch.cuda.stream(s):
                with graph_capture(g, s):
                    for _ in range(k):
                        self._step()
        except Exception as e:
            if os.environ.get("DDL_GRAPHS_STRICT") == "1":
                raise
            print(f"[ddl] batched replica hipGraph capture disabled: {type(e).__name__}: {e}", flush=True)
            torch.cuda.synchronize(self.dev)
            return False
        torch.cuda.current_stream(self.dev).wait_stream(s)
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
