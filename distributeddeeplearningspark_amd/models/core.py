"""Keras-compatible model API (``Sequential``, layers, ``compile/fit/train_on_batch/
predict/get_weights/set_weights/summary/to_json``) on top of the MI355X op layer.

The reference builds Keras 2 ``Sequential`` models (``ddl_mnist_aztk.py:180-199``,
``ddl_nyiso_aztk.py:201-204,249-252``) and hands them to dist-keras trainers that
serialise them as ``{'model': to_json(), 'weights': get_weights()}``.  This module
keeps that surface: Keras weight layouts/ordering in ``get_weights`` and a
Keras-shaped JSON config, while the storage underneath is the flat parameter arena
(``params.py``) and every op dispatches to the HIP kernels on the GPU.

Activations are NHWC; on the GPU they are bf16 with fp32 master weights.
"""
from __future__ import annotations

import json
import math
import time
from typing import Any, Sequence

import numpy as np
import torch

from . import optimizers as optim_mod
from .params import Param, ParamArena, to_numpy

_LAYER_TYPES: dict[str, type] = {}
_UNIT_SEEDS: dict = {}  # (device, dtype, shape) -> ones: the backward seed of training steps
_NAME_COUNTS: dict[str, int] = {}


FUSE_CONVBN = True  # Sequential Conv2D -> BN (-> ReLU) as one fused training node (tests compare with False)


def _auto_name(prefix: str) -> str:
    n = _NAME_COUNTS.get(prefix, 0) + 1
    _NAME_COUNTS[prefix] = n
    return f"{prefix}_{n}"


def _snake(name: str) -> str:
    out = []
    for i, ch in enumerate(name):
        if ch.isupper() and i and not name[i - 1].isupper():
            out.append("_")
        out.append(ch.lower())
    return "".join(out)


class Layer:
    """Base layer.  Subclasses define ``build`` (create params with ``add_weight``),
    ``call`` and ``compute_output_shape``; shapes exclude the batch dimension."""

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        _LAYER_TYPES[cls.__name__] = cls

    def __init__(self, name: str | None = None, input_shape=None, input_dim=None, trainable: bool = True,
                 batch_input_shape=None, **kwargs):
        if kwargs:
            unknown = set(kwargs) - {"dtype", "weights"}
            if unknown:
                raise TypeError(f"{type(self).__name__}: unexpected arguments {sorted(unknown)}")
        self.name = name or _auto_name(_snake(type(self).__name__))
        if batch_input_shape is not None:
            input_shape = tuple(batch_input_shape[1:])
        if input_shape is None and input_dim is not None:
            input_shape = (int(input_dim),)
        self._input_shape_arg = tuple(input_shape) if input_shape is not None else None
        self.trainable = trainable
        self.built = False
        self._params: list[Param] = []
        self._states: dict[str, torch.Tensor] = {}
        self.input_shape = None
        self.output_shape = None
        self.grad_hook = None  # set by the data-parallel engine (fires when this layer's grads are final)
        self._initial_weights = kwargs.get("weights")

    # ------------------------------------------------------------------ params
    def add_weight(self, name: str, shape, init, trainable: bool = True, pad=None) -> Param:
        p = Param(f"{self.name}/{name}", shape, init, trainable, pad=pad)
        self._params.append(p)
        return p

    def add_state(self, name: str, value: torch.Tensor) -> torch.Tensor:
        self._states[name] = value.to(torch.float32)
        return self._states[name]

    def sublayers(self) -> list["Layer"]:
        return []

    def all_params(self) -> list[Param]:
        out = list(self._params)
        for l in self.sublayers():
            out.extend(l.all_params())
        return out

    def all_layers(self) -> list["Layer"]:
        out = [self]
        for l in self.sublayers():
            out.extend(l.all_layers())
        return out

    def count_params(self) -> int:
        return sum(p.numel for p in self.all_params())

    # ------------------------------------------------------------------ lifecycle
    def build(self, input_shape):
        self.built = True

    def ensure_built(self, input_shape):
        if not self.built:
            self.input_shape = tuple(input_shape)
            self.build(tuple(input_shape))
            self.built = True
            self.output_shape = tuple(self.compute_output_shape(tuple(input_shape)))
        return self.output_shape

    def compute_output_shape(self, input_shape):
        return input_shape

    def call(self, x, training: bool = False):
        raise NotImplementedError

    def __call__(self, x, training: bool = False):
        return self.call(x, training)

    def states_to(self, device):
        for k, v in list(self._states.items()):
            self._states[k] = v.to(device)
        for l in self.sublayers():
            l.states_to(device)

    # ------------------------------------------------------------------ keras weights
    def keras_weight_params(self) -> list:
        """Ordered entries of Keras ``get_weights()``: Param objects or state names."""
        return list(self._params)

    def get_keras_weights(self) -> list[np.ndarray]:
        out = []
        for e in self.keras_weight_params():
            if isinstance(e, Param):
                out.append(e.to_keras(to_numpy(e.master)))
            else:
                out.append(to_numpy(self._states[e]))
        return out

    def set_keras_weights(self, ws: Sequence[np.ndarray]):
        ents = self.keras_weight_params()
        if len(ws) != len(ents):
            raise ValueError(f"{self.name}: expected {len(ents)} weight arrays, got {len(ws)}")
        for e, w in zip(ents, ws):
            if isinstance(e, Param):
                arr = np.asarray(e.from_keras(np.asarray(w, dtype=np.float32)), dtype=np.float32).reshape(e.shape)
                if e.master is None:
                    e._initial = arr
                else:
                    with torch.no_grad():
                        e.master.copy_(torch.from_numpy(arr))
            else:
                self._states[e].copy_(torch.as_tensor(np.asarray(w), dtype=torch.float32))

    # ------------------------------------------------------------------ config
    def get_config(self) -> dict:
        cfg = {"name": self.name, "trainable": self.trainable}
        if self._input_shape_arg is not None:
            cfg["batch_input_shape"] = [None, *self._input_shape_arg]
        return cfg

    @classmethod
    def from_config(cls, cfg: dict):
        cfg = dict(cfg)
        return cls(**cfg)

    def __repr__(self):
        return f"<{type(self).__name__} {self.name}>"


def layer_from_config(d: dict) -> Layer:
    cls = _LAYER_TYPES.get(d["class_name"])
    if cls is None:
        raise ValueError(f"unknown layer class {d['class_name']!r}")
    return cls.from_config(d["config"])


# =========================================================================================
#                                         Model
# =========================================================================================
_LOSS_ALIASES = {
    "mse": "mean_squared_error",
    "mae": "mean_absolute_error",
    "categorical_crossentropy": "categorical_crossentropy",
    "sparse_categorical_crossentropy": "sparse_categorical_crossentropy",
    "binary_crossentropy": "binary_crossentropy",
    "mean_squared_error": "mean_squared_error",
    "mean_absolute_error": "mean_absolute_error",
}


class Model(Layer):
    """A trainable network: owns the parameter arena, optimizer and loss."""

    def __init__(self, name=None, **kw):
        super().__init__(name=name, **kw)
        self.arena: ParamArena | None = None
        self.device = torch.device("cpu")
        self.compute_dtype = torch.float32
        self.optimizer = None
        self.loss = None
        self.metrics: list = []
        self.history: list[float] = []
        self.seed = 0
        # uint8 NHWC image inputs are normalised on the device by to_input:
        # (x - mean[c]) / std[c]; default mean 0 / std 255 (Keras' rescale=1/255)
        self.input_mean: tuple | None = None
        self.input_std: tuple | None = None

    # ---------------------------------------------------------------- placement
    def build_model(self):
        raise NotImplementedError

    def place(self, device=None, dtype=None, seed: int | None = None):
        """Allocate the flat parameter arena on ``device`` (bf16 compute on GPU)."""
        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        device = torch.device(device)
        self.build_model()
        if dtype is None:
            dtype = torch.bfloat16 if device.type == "cuda" and not self._keeps_fp32() else torch.float32
        old = None
        if self.arena is not None:
            old = self.arena.get_flat().detach().cpu()  # canonical: the new arena may pad differently
        params = self.all_params()
        self.arena = ParamArena(params, device, dtype, seed=self.seed if seed is None else seed)
        if old is not None and old.numel() == self.arena.canon_numel:
            self.arena.set_flat(old)
        self.states_to(device)
        self.device, self.compute_dtype = device, dtype
        if self.optimizer is not None:
            self.optimizer.bind(self.arena)
        return self

    @property
    def graph_capturable(self) -> bool:
        """False when the model draws host-side per-step state a replayed hipGraph would freeze (BERT's
        step-seeded dropout sets it).  Dropout layers do not: inside a capture their kernels mix a device step
        counter into the seed, which every captured step ticks (``ops/act.py dropout_step_counter``)."""
        if "_graph_capturable" in self.__dict__:
            return self.__dict__["_graph_capturable"]
        return True

    @graph_capturable.setter
    def graph_capturable(self, v: bool):
        self.__dict__["_graph_capturable"] = bool(v)

    def _keeps_fp32(self) -> bool:
        """Recurrent models train in fp32 on the GPU too: they are the reference's Keras
        regressors (fp32 GRU/LSTM, ``ddl_nyiso_aztk.py:201-203``), tiny and latency-bound, so
        bf16 would cost accuracy (MAPE) without buying any speed."""
        from .layers import _Recurrent

        return any(isinstance(l, _Recurrent) for l in self.all_layers())

    def _ensure_placed(self):
        if self.arena is None:
            self.place()

    # ---------------------------------------------------------------- compile / train
    def compile(self, optimizer="sgd", loss="mean_squared_error", metrics=None, **kw):
        self.optimizer = optim_mod.get(optimizer)
        if isinstance(loss, str):
            if loss not in _LOSS_ALIASES:
                raise ValueError(f"unknown loss {loss!r}")
            loss = _LOSS_ALIASES[loss]
        self.loss = loss
        self.metrics = list(metrics or [])
        if self.arena is not None:
            self.optimizer.bind(self.arena)
        return self

    def to_input(self, x) -> torch.Tensor:
        if isinstance(x, np.ndarray):
            x = torch.from_numpy(np.ascontiguousarray(x))
        x = torch.as_tensor(x)
        if x.is_floating_point():
            return x.to(self.device, self.compute_dtype, non_blocking=True)
        x = x.to(self.device, non_blocking=True)
        if self.takes_integer_inputs():
            return x  # token ids (an Embedding first layer)
        if x.dtype == torch.uint8 and x.dim() == 4:
            # uint8 NHWC pixels: (x - input_mean) / input_std per channel, or x / 255 when the model
            # declares no normalisation (the Keras-style default for image batches)
            return self.normalize_images(x)
        # any other integer / bool feature column (2-D / 3-D: counts, ids, flags): its values, in the
        # compute dtype (the Dense / Conv kernels take floating inputs only)
        return x.to(self.compute_dtype)

    def takes_integer_inputs(self) -> bool:
        """True when the first layer consumes integer ids (``Embedding``)."""
        subs = self.sublayers()
        return bool(subs) and type(subs[0]).__name__ == "Embedding"

    def normalize_images(self, x_u8: torch.Tensor) -> torch.Tensor:
        """uint8 NHWC -> compute dtype, (x - mean) / std per channel: one HIP pass on the GPU
        (``normalize_u8``, the kernel the ingest feeder uses), torch on the CPU."""
        from ..ops._native import C, use_native

        c = x_u8.shape[-1]
        key = (str(x_u8.device), c, self.input_mean, self.input_std)
        cache = self.__dict__.setdefault("_norm_cache", {})
        if key not in cache:  # device-resident constants: no host->device copy per batch
            mean = torch.tensor((self.input_mean or (0.0,) * c)[:c], dtype=torch.float32, device=x_u8.device)
            std = torch.tensor((self.input_std or (255.0,) * c)[:c], dtype=torch.float32, device=x_u8.device)
            cache[key] = (mean, std, (1.0 / std).contiguous())
        mean, std, invstd = cache[key]
        if use_native(x_u8):
            out = torch.empty(x_u8.shape, dtype=self.compute_dtype, device=x_u8.device)
            C().normalize_u8(x_u8.contiguous(), out, mean, invstd, c, c)
            return out
        return ((x_u8.to(torch.float32) - mean) / std).to(self.compute_dtype)

    def to_target(self, y) -> torch.Tensor:
        if isinstance(y, np.ndarray):
            y = torch.from_numpy(np.ascontiguousarray(y))
        y = torch.as_tensor(y)
        return y.to(self.device, non_blocking=True)

    # subclasses: forward(x, training, logits=False)
    def forward(self, x, training=False, logits=False):
        raise NotImplementedError

    def call(self, x, training=False):
        return self.forward(x, training)

    def ends_with_softmax(self) -> bool:
        return False

    def compute_loss(self, x, y, training=True):
        from ..ops import loss as L

        name = self.loss
        if callable(name):
            return name(self.forward(x, training), y)
        if name in ("categorical_crossentropy", "sparse_categorical_crossentropy") and self.ends_with_softmax():
            logits = self.forward(x, training, logits=True)
            logits = logits.reshape(logits.shape[0], -1)
            if name == "sparse_categorical_crossentropy" or not y.is_floating_point():
                return L.softmax_cross_entropy(logits, labels=y.reshape(-1).long())
            return L.softmax_cross_entropy(logits, probs=y.reshape(logits.shape))
        out = self.forward(x, training).float()
        yy = y.float().reshape(out.shape)
        if name == "mean_squared_error":
            return L.mean_squared_error(out, yy)
        if name == "mean_absolute_error":
            return L.mean_absolute_error(out, yy)
        if name == "binary_crossentropy":
            return L.binary_crossentropy(out, yy)
        if name == "categorical_crossentropy":
            return L.categorical_crossentropy_probs(out, yy)
        if name == "sparse_categorical_crossentropy":  # probability output (no fused softmax): HIP on the GPU
            return L.prob_cross_entropy(out.reshape(out.shape[0], -1), labels=y.reshape(-1))
        raise ValueError(f"unsupported loss {name!r}")

    def backward_step(self, x, y):
        """zero grads -> forward -> loss -> backward (grads land in the arena). Returns loss tensor."""
        from ..ops.norm import reset_workspaces

        from ..ops import derived

        self._ensure_placed()
        reset_workspaces(self.device, extra=self.arena.zero_grad(defer=True))  # one zeroing launch
        derived.begin_step(self)  # weight-derived filters: one launch per step (ops/derived.py)
        try:
            loss = self.compute_loss(x, y, training=True)
            self.backward_unit(loss)
        finally:
            derived.end_step()
        return loss

    def backward_unit(self, loss):
        """``loss.backward()`` with the model (and the loss nodes, ``ops.loss.unit_seed``) told that the
        seed gradient is exactly 1: they hand out their stored gradients without applying it, and the
        seed itself is a cached device constant (no fill launch per step)."""
        from ..ops import loss as loss_ops
        from ..ops.streams import join

        key = (loss.device, loss.dtype, loss.shape)
        one = _UNIT_SEEDS.get(key)
        if one is None:
            one = _UNIT_SEEDS[key] = torch.ones(loss.shape, dtype=loss.dtype, device=loss.device)
        self._unit_loss_grad = True
        loss_ops._UNIT_SEED[0] = loss.grad_fn
        try:
            loss.backward(one)
        finally:
            self._unit_loss_grad = False
            loss_ops._UNIT_SEED[0] = None
        join(self.device)  # side-stream weight gradients (ops/streams.py) land before anyone reads them

    def train_on_batch(self, x, y, grad_sync=None, grad_scale: float = 1.0) -> float:
        if self.optimizer is None:
            raise RuntimeError("call compile() before training")
        self._ensure_placed()
        if self.optimizer.arena is not self.arena:
            self.optimizer.bind(self.arena)
        x, y = self.to_input(x), self.to_target(y)
        loss = self.backward_step(x, y)
        if grad_sync is not None:
            grad_scale = grad_sync(self.arena) * grad_scale
        self.optimizer.step(grad_scale)
        return float(loss.detach())

    def fit(self, x, y, batch_size=32, epochs=1, verbose=0, shuffle=True, drop_last=False):
        x = np.asarray(x)
        y = np.asarray(y)
        n = x.shape[0]
        rng = np.random.default_rng(self.seed)
        hist = []
        for ep in range(epochs):
            idx = rng.permutation(n) if shuffle else np.arange(n)
            losses = []
            stop = n - (n % batch_size) if drop_last else n
            for b in range(0, stop, batch_size):
                sel = idx[b : b + batch_size]
                losses.append(self.train_on_batch(x[sel], y[sel]))
            hist.append(float(np.mean(losses)) if losses else float("nan"))
            if verbose:
                print(f"Epoch {ep + 1}/{epochs} - loss: {hist[-1]:.4f}")
        self.history.extend(hist)
        return {"loss": hist}

    @torch.no_grad()
    def predict(self, x, batch_size=256) -> np.ndarray:
        self._ensure_placed()
        x = np.asarray(x) if not isinstance(x, torch.Tensor) else x
        outs = []
        for b in range(0, x.shape[0], batch_size):
            xb = self.to_input(x[b : b + batch_size])
            outs.append(self.forward(xb, training=False).float().cpu())
        if not outs:
            return np.zeros((0,) + tuple(self.output_shape or ()), dtype=np.float32)
        return torch.cat(outs).numpy()

    @torch.no_grad()
    def evaluate(self, x, y, batch_size=256) -> float:
        self._ensure_placed()
        tot, cnt = 0.0, 0
        for b in range(0, len(x), batch_size):
            xb, yb = self.to_input(np.asarray(x[b : b + batch_size])), self.to_target(np.asarray(y[b : b + batch_size]))
            tot += float(self.compute_loss(xb, yb, training=False)) * xb.shape[0]
            cnt += xb.shape[0]
        return tot / max(cnt, 1)

    # ---------------------------------------------------------------- weights / serialisation
    def weight_layers(self) -> list[Layer]:
        return [l for l in self.all_layers() if l is not self and (l._params or l._states)]

    def get_weights(self) -> list[np.ndarray]:
        self.build_model()
        if self.arena is None:  # materialise the initial weights (host memory, no GPU touch)
            self.place("cpu")
        out = []
        for l in self.weight_layers():
            if l.keras_weight_params():
                out.extend(l.get_keras_weights())
        return out

    def set_weights(self, weights: Sequence[np.ndarray]):
        self.build_model()
        weights = list(weights)
        i = 0
        for l in self.weight_layers():
            n = len(l.keras_weight_params())
            if n:
                l.set_keras_weights(weights[i : i + n])
                i += n
        if i != len(weights):
            raise ValueError(f"set_weights: expected {i} arrays, got {len(weights)}")
        if self.arena is not None:
            self.arena.sync_compute()

    def get_flat_weights(self) -> torch.Tensor:
        self._ensure_placed()
        return self.arena.get_flat()

    def to_json(self) -> str:
        d = {"class_name": type(self).__name__, "config": self.get_config(),
             "backend": "distributeddeeplearningspark_amd", "keras_version": "2.1.6"}
        if self.input_mean is not None or self.input_std is not None:
            d["input_normalization"] = {"mean": self.input_mean, "std": self.input_std}
        return json.dumps(d)

    def summary(self, print_fn=print):
        self.build_model()
        line = "_" * 65
        print_fn(line)
        print_fn(f"{'Layer (type)':<29}{'Output Shape':<25}{'Param #':<11}")
        print_fn("=" * 65)
        rows = self.summary_rows()
        for i, (nm, shp, cnt) in enumerate(rows):
            print_fn(f"{nm:<29}{shp:<25}{cnt:<11}")
            print_fn("=" * 65 if i == len(rows) - 1 else line)
        total = self.count_params()
        print_fn(f"Total params: {total:,}")
        print_fn(f"Trainable params: {total:,}")
        print_fn("Non-trainable params: 0")
        print_fn(line)

    def summary_rows(self):
        rows = []
        for l in self.sublayers():
            shp = "(None, " + ", ".join(str(s) for s in (l.output_shape or ())) + ")"
            if l.output_shape is not None and len(l.output_shape) == 1:
                shp = f"(None, {l.output_shape[0]})"
            rows.append((f"{l.name} ({type(l).__name__})", shp, l.count_params()))
        return rows


class Sequential(Model):
    """Keras ``Sequential``: ``add`` layers, the first carries ``input_shape``."""

    def __init__(self, layers: Sequence[Layer] | None = None, name=None, **kw):
        super().__init__(name=name or _auto_name("sequential"), **kw)
        self.layers: list[Layer] = []
        for l in layers or []:
            self.add(l)

    def add(self, layer: Layer):
        if self.arena is not None:
            raise RuntimeError("cannot add layers after the model was placed")
        self.layers.append(layer)
        self.built = False

    def sublayers(self):
        return list(self.layers)

    def build_model(self):
        if self.built:
            return
        if not self.layers:
            raise ValueError("empty Sequential model")
        shape = self.layers[0]._input_shape_arg or self._input_shape_arg
        if shape is None:
            raise ValueError("the first layer needs input_shape=")
        self.input_shape = tuple(shape)
        for l in self.layers:
            shape = l.ensure_built(shape)
        self.output_shape = tuple(shape)
        self.built = True

    def ends_with_softmax(self) -> bool:
        last = self.layers[-1] if self.layers else None
        return getattr(last, "activation_name", None) == "softmax"

    def forward(self, x, training=False, logits=False):
        """Runs the layers with graph-level fusions: Conv2D/Dense + Activation('relu') ->
        ReLU epilogue; Conv2D -> BatchNormalization -> relu: BN statistics accumulated in
        the conv epilogue and ReLU fused into the BN apply; final softmax skipped when the
        loss is the fused softmax-cross-entropy (``logits=True``)."""
        from ..ops._native import use_native
        from ..ops.norm import new_stats_workspace
        from .layers import Activation, BatchNormalization, Conv2D, Dense, MaxPooling2D

        L = self.layers
        n = len(L)
        i = 0
        while i < n:
            l = L[i]
            nxt = L[i + 1] if i + 1 < n else None
            nxt2 = L[i + 2] if i + 2 < n else None
            if logits and i == n - 1 and getattr(l, "activation_name", None) == "softmax":
                if hasattr(l, "supports_skip"):
                    x = l.call(x, training, skip_activation=True)
                break
            relu_next = isinstance(nxt, Activation) and nxt.activation_name == "relu"
            if isinstance(l, Conv2D) and l.activation_name == "linear" and isinstance(nxt, BatchNormalization):
                relu2 = isinstance(nxt2, Activation) and nxt2.activation_name == "relu"
                unit = self._convbn_unit(l, nxt, x) if (training and use_native(x)) else None
                if unit is not None:
                    # conv + BN (+ReLU) as ONE autograd node with a hand-scheduled backward
                    # (ops/fused_blocks.py: half the Python / autograd work per layer)
                    from ..ops.fused_blocks import convbn_relu, convbn_relu_pool

                    nxt3 = L[i + 3] if i + 3 < n else None
                    if (relu2 and isinstance(nxt3, MaxPooling2D) and nxt3.pool_size == (2, 2)
                            and nxt3.strides == (2, 2) and nxt3.padding == "valid"):
                        # ... and the 2x2 max pool behind it: the pool applies BN + ReLU as it loads
                        y = convbn_relu_pool(unit, x, l.kernel.data)
                        if y is not None:
                            x = y
                            i += 4
                            continue
                    x = convbn_relu(unit, x, l.kernel.data, relu=relu2)
                    i += 3 if relu2 else 2
                    continue
                stats = new_stats_workspace(l.filters, x.device) if (training and use_native(x)) else None
                y = l.call(x, training, stats=stats)
                relu2 = isinstance(nxt2, Activation) and nxt2.activation_name == "relu"
                x = nxt.call(y, training, relu=relu2, stats=stats)
                i += 3 if relu2 else 2
                continue
            if relu_next and isinstance(l, (Conv2D, Dense)) and l.activation_name == "linear":
                x = l.call(x, training, relu=True)
                i += 2
                continue
            if relu_next and isinstance(l, BatchNormalization):
                x = l.call(x, training, relu=True)
                i += 2
                continue
            x = l.call(x, training)
            i += 1
        return x

    def _convbn_unit(self, conv, bn, x):
        """The (conv, BN) pair as a ``fused_blocks`` unit when the fused training node applies: no conv
        bias, stride 1 or an even split of "same" padding (no explicit pre-pad), dilation 1, both
        trainable; ``FUSE_CONVBN = False`` keeps the two-node path."""
        if not FUSE_CONVBN or conv.bias is not None or conv.dilation_rate != (1, 1):
            return None
        if not (conv.trainable and bn.trainable and bn.gamma is not None and bn.beta is not None):
            return None
        (ph, pw), extra = conv._pads(x.shape[1], x.shape[2])
        if extra is not None:
            return None
        cache = self.__dict__.setdefault("_convbn_units", {})
        key = (id(conv), ph, pw)
        u = cache.get(key)
        if u is None:
            u = cache[key] = _ConvBNUnit(conv, bn, (ph, pw))
        return u

    def get_config(self):
        return {"name": self.name, "layers": [{"class_name": type(l).__name__, "config": l.get_config()}
                                              for l in self.layers]}

    @classmethod
    def from_config(cls, cfg):
        m = cls(name=cfg.get("name"))
        for d in cfg["layers"]:
            m.add(layer_from_config(d))
        return m


def model_from_json(s: str) -> Model:
    d = json.loads(s)
    cls = _LAYER_TYPES.get(d["class_name"])
    if cls is None:
        raise ValueError(f"unknown model class {d['class_name']!r}")
    m = cls.from_config(d["config"])
    norm = d.get("input_normalization")
    if norm:
        m.input_mean = None if norm.get("mean") is None else tuple(norm["mean"])
        m.input_std = None if norm.get("std") is None else tuple(norm["std"])
    return m


class _PaddedConv:
    """View of a Conv2D layer with its padding resolved to a (ph, pw) tuple (every other attribute,
    the gradient hook included, read through to the layer at use time)."""

    def __init__(self, conv, pads):
        self.__dict__["_conv"] = conv
        self.__dict__["padding"] = pads

    def __getattr__(self, name):
        return getattr(self.__dict__["_conv"], name)


class _ConvBNUnit:
    """(conv, BN) pair in the shape ``ops.fused_blocks`` expects of a ResNet ConvBN unit."""

    def __init__(self, conv, bn, pads):
        self.conv = _PaddedConv(conv, pads)
        self.bn = bn

