"""Keras-style optimizers on the flat parameter arena (``worker_optimizer='adam'`` etc.).

Defaults follow Keras 2 (the reference's per-worker optimizers, ``ddl_mnist_aztk.py:195``,
``ddl_nyiso_aztk.py:207,255``): Adam(lr=1e-3, eps=1e-7, Keras epsilon placement),
Adagrad(lr=1e-2, eps=1e-7), RMSprop(lr=1e-3, rho=0.9), SGD(lr=1e-2).
Each optimizer's ``step`` is ONE kernel launch over the whole model on the GPU.
"""
from __future__ import annotations

import torch

from ..ops import optim as K


class Optimizer:
    name = "optimizer"

    def __init__(self, lr: float, weight_decay: float = 0.0, clipnorm: float | None = None):
        self.lr = float(lr)
        self.weight_decay = float(weight_decay)
        self.clipnorm = clipnorm
        self.iterations = 0
        self.arena = None
        self.state: dict[str, torch.Tensor] = {}
        self.device_step: torch.Tensor | None = None  # set for graph capture (models/step.py)
        self.tick_ctr: torch.Tensor | None = None  # int32 workgroup counter of the fused tick (Adam)

    def bind(self, arena):
        self.arena = arena
        self.iterations = 0
        self.device_step = None
        self._alloc()
        return self

    def _alloc(self):
        pass

    def _zeros(self):
        return torch.zeros_like(self.arena.master)

    def get_config(self):
        return {"name": self.name, "lr": self.lr, "weight_decay": self.weight_decay}

    def state_dict(self):
        """Iterations + the flat state slots in the arena's canonical layout (params.py)."""
        conv = self.arena.to_canonical if self.arena is not None else (lambda t: t)
        return {"iterations": self.iterations, **{k: conv(v.detach()).cpu() for k, v in self.state.items()}}

    def load_state_dict(self, sd):
        self.iterations = int(sd.get("iterations", 0))
        for k, v in sd.items():
            if k in self.state:
                v = v.to(self.state[k].device)
                if self.arena is not None and self.arena.padded:
                    # state_dict() always saves the canonical layout; the two layouts can have the same
                    # numel (padding inside the ALIGN rounding) while placing values differently
                    if v.numel() != self.arena.canon_numel:
                        raise ValueError(f"optimizer slot {k!r}: {v.numel()} elements, the canonical layout "
                                         f"has {self.arena.canon_numel}")
                    v = self.arena.from_canonical(v)
                self.state[k].copy_(v)
        if self.device_step is not None:
            self.device_step.fill_(float(self.iterations))

    # ---------------------------------------------------------------- graph capture
    def enable_device_step(self):
        """Keep the step counter on the GPU (needed once a step is replayed from a hipGraph:
        host scalars baked into a captured launch would never change)."""
        if self.device_step is None and self.arena is not None and self.arena.master.is_cuda:
            self.device_step = torch.full((1,), float(self.iterations), dtype=torch.float32,
                                          device=self.arena.master.device)
            self.tick_ctr = torch.zeros(1, dtype=torch.int32, device=self.arena.master.device)

    def _grad_scale(self, grad_scale):
        if self.clipnorm is None:
            return grad_scale
        g = self.arena.grad
        norm = float(torch.linalg.vector_norm(g)) * grad_scale
        if norm > self.clipnorm:
            return grad_scale * self.clipnorm / (norm + 1e-6)
        return grad_scale

    def step(self, grad_scale: float = 1.0):
        gs = self.begin_step(grad_scale)
        self.apply_range(0, self.arena.numel, gs)

    # ---------------------------------------------------------------- ranged steps
    # The data-parallel engine updates the arena bucket by bucket, each slice as soon as its
    # all-reduce has landed, so the optimizer sweep over the early buckets runs under the
    # reduction of the last one (parallel/ddp.py).  One logical step = begin_step + apply_range
    # over a partition of [0, numel); the update of every element is identical to ``step``.
    def begin_step(self, grad_scale: float = 1.0) -> float:
        """Advance the step counter (host and device) once; returns the effective grad scale."""
        self.iterations += 1
        if self.device_step is not None and self._device_tick:
            K.step_tick(self.device_step)
        return self._grad_scale(grad_scale)

    def apply_range(self, lo: int, hi: int, gs: float):
        """Update arena elements [lo, hi) (lo, hi multiples of the arena alignment)."""
        if hi <= lo:
            return
        a = self.arena
        sl = slice(int(lo), int(hi))
        w16 = None if a.compute is a.master else a.compute[sl]
        self._apply(a.master[sl], a.grad[sl], w16, gs, {k: v[sl] for k, v in self.state.items()})

    def captured_update(self, gs: float = 1.0, zero_grads: bool = False):
        """The device-side part of one step (step-counter tick + full update) for a hipGraph
        capture; the host counter is advanced per replay by the caller (models/step.py).

        ``zero_grads``: the caller captures another step right after this one — optimizers that can
        zero the gradients as they consume them do so, and the arena skips that step's zero_grad fill
        (``ParamArena.grads_zeroed``).  Adam also advances the device step counter inside its own
        launch (no step_tick)."""
        a = self.arena
        if self._fused_update(gs, zero_grads):
            a.grads_zeroed = zero_grads
            return
        if self.device_step is not None and self._device_tick:
            K.step_tick(self.device_step)
        self.apply_range(0, a.numel, gs)

    def _fused_update(self, gs: float, zero_grads: bool) -> bool:
        return False

    @property
    def ranged_ok(self) -> bool:
        """A global gradient norm (clipnorm) needs every bucket reduced before any update."""
        return self.clipnorm is None

    _device_tick = False  # optimizers whose kernels read the device step counter (Adam family)

    def _apply(self, w, g, w16, gs, st):
        raise NotImplementedError


class SGD(Optimizer):
    name = "sgd"

    def __init__(self, lr=0.01, momentum=0.0, nesterov=False, dampening=0.0, weight_decay=0.0, clipnorm=None):
        super().__init__(lr, weight_decay, clipnorm)
        self.momentum, self.nesterov, self.dampening = float(momentum), bool(nesterov), float(dampening)

    def _alloc(self):
        if self.momentum:
            self.state["momentum"] = self._zeros()

    def _apply(self, w, g, w16, gs, st):
        K.sgd_(w, g, st.get("momentum"), w16, lr=self.lr, momentum=self.momentum, dampening=self.dampening,
               weight_decay=self.weight_decay, nesterov=self.nesterov, grad_scale=gs)

    def get_config(self):
        return {**super().get_config(), "momentum": self.momentum, "nesterov": self.nesterov}


class Adam(Optimizer):
    name = "adam"

    def __init__(self, lr=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-7, weight_decay=0.0, decoupled=False,
                 keras_eps=True, clipnorm=None):
        super().__init__(lr, weight_decay, clipnorm)
        self.b1, self.b2, self.eps = float(beta_1), float(beta_2), float(epsilon)
        self.decoupled, self.keras_eps = bool(decoupled), bool(keras_eps)

    def _alloc(self):
        self.state["m"] = self._zeros()
        self.state["v"] = self._zeros()

    _device_tick = True

    def _apply(self, w, g, w16, gs, st, tick_ctr=None, zero_grad=False):
        K.adam_(w, g, st["m"], st["v"], w16, lr=self.lr, beta1=self.b1, beta2=self.b2, eps=self.eps,
                weight_decay=self.weight_decay, decoupled=self.decoupled, keras_eps=self.keras_eps,
                step=self.iterations, grad_scale=gs, device_step=self.device_step, tick_ctr=tick_ctr,
                zero_grad=zero_grad)

    def _fused_update(self, gs, zero_grads):
        """One launch: tick + update (+ gradient zeroing) over the whole arena."""
        a = self.arena
        if self.device_step is None or self.tick_ctr is None or not a.master.is_cuda:
            return False
        self._apply(a.master, a.grad, None if a.compute is a.master else a.compute, gs, self.state,
                    tick_ctr=self.tick_ctr, zero_grad=zero_grads)
        return True

    def get_config(self):
        return {**super().get_config(), "beta_1": self.b1, "beta_2": self.b2, "epsilon": self.eps}


class AdamW(Adam):
    name = "adamw"

    def __init__(self, lr=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-8, weight_decay=0.01, clipnorm=None):
        super().__init__(lr, beta_1, beta_2, epsilon, weight_decay, decoupled=True, keras_eps=False,
                         clipnorm=clipnorm)


class Adagrad(Optimizer):
    name = "adagrad"

    def __init__(self, lr=0.01, epsilon=1e-7, weight_decay=0.0, clipnorm=None):
        super().__init__(lr, weight_decay, clipnorm)
        self.eps = float(epsilon)

    def _alloc(self):
        self.state["acc"] = self._zeros()

    def _apply(self, w, g, w16, gs, st):
        K.adagrad_(w, g, st["acc"], w16, lr=self.lr, eps=self.eps, weight_decay=self.weight_decay,
                   grad_scale=gs)


class RMSprop(Optimizer):
    name = "rmsprop"

    def __init__(self, lr=0.001, rho=0.9, epsilon=1e-7, weight_decay=0.0, clipnorm=None):
        super().__init__(lr, weight_decay, clipnorm)
        self.rho, self.eps = float(rho), float(epsilon)

    def _alloc(self):
        self.state["acc"] = self._zeros()

    def _apply(self, w, g, w16, gs, st):
        K.rmsprop_(w, g, st["acc"], w16, lr=self.lr, rho=self.rho, eps=self.eps,
                   weight_decay=self.weight_decay, grad_scale=gs)


_BY_NAME = {"sgd": SGD, "adam": Adam, "adamw": AdamW, "adagrad": Adagrad, "rmsprop": RMSprop}


def get(spec) -> Optimizer:
    """Resolve a Keras optimizer spec: a name (``'adam'``), a config dict or an instance."""
    if isinstance(spec, Optimizer):
        return spec
    if isinstance(spec, str):
        key = spec.lower()
        if key not in _BY_NAME:
            raise ValueError(f"unknown optimizer {spec!r}; known: {sorted(_BY_NAME)}")
        return _BY_NAME[key]()
    if isinstance(spec, dict):
        cfg = dict(spec)
        name = cfg.pop("name")
        return _BY_NAME[name.lower()](**cfg)
    raise TypeError(f"bad optimizer spec {spec!r}")


def clone(opt: Optimizer) -> Optimizer:
    """Fresh optimizer with the same hyper-parameters (worker-local optimizer state)."""
    return get(opt.get_config()) if isinstance(opt, Optimizer) else get(opt)
