"""Keras-compatible layers (the set the reference uses plus what the north-star models need).

Reference layer usage: ``Conv2D / Activation / MaxPooling2D / Flatten / Dense``
(``ddl_mnist_aztk.py:180-192``), ``GRU`` (``ddl_nyiso_aztk.py:201-203``), ``LSTM``
(``ddl_nyiso_aztk.py:249-251``).  Weight layouts returned by ``get_weights`` are Keras'
(Conv2D kernel [kh,kw,cin,cout], Dense kernel [in,out], GRU/LSTM kernel [in,nG*H],
recurrent_kernel [H,nG*H], bias [nG*H]); internal layouts are MFMA-friendly
(Conv2D [cout,kh,kw,cin], Dense [out,in]).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

from ..ops import act as act_ops
from ..ops import conv as conv_ops
from ..ops import linear as linear_ops
from ..ops import norm as norm_ops
from ..ops import pool as pool_ops
from ..ops import rnn as rnn_ops
from . import params as P
from .core import Layer

# activation names of the Keras layer set: HIP kernels on the GPU (ops/act.py), torch on the CPU
_ACTS = (None, "linear") + act_ops.ACT_NAMES + ("softmax",)


def _act_name(a):
    if a is None:
        return "linear"
    if callable(a):
        return getattr(a, "__name__", "custom")
    if a not in _ACTS:
        raise ValueError(f"unknown activation {a!r}")
    return a


def apply_activation(name, x):
    return act_ops.activation(x, name)


def _pair(v):
    return (int(v), int(v)) if isinstance(v, (int, np.integer)) else tuple(int(t) for t in v)


def _r8(n: int) -> int:
    """Storage width of a GEMM operand dimension: whole 16-B bf16 vectors (``params.Param(pad=)``)."""
    return -(-int(n) // 8) * 8


class Activation(Layer):
    def __init__(self, activation, **kw):
        super().__init__(**kw)
        self.activation_name = _act_name(activation)

    supports_skip = True

    def call(self, x, training=False, skip_activation=False):
        return x if skip_activation else apply_activation(self.activation_name, x)

    def get_config(self):
        return {**super().get_config(), "activation": self.activation_name}


class Dense(Layer):
    def __init__(self, units, activation=None, use_bias=True, kernel_initializer="glorot_uniform", **kw):
        super().__init__(**kw)
        self.units = int(units)
        self.activation_name = _act_name(activation)
        self.use_bias = use_bias
        self.kernel_initializer = kernel_initializer
        self.fuse_relu = False  # set by Sequential when followed by Activation('relu')

    supports_skip = True

    def build(self, input_shape):
        fin = int(input_shape[-1])
        init = P.he_normal(fin) if self.kernel_initializer == "he_normal" else P.glorot_uniform(fin, self.units)
        self.kernel = self.add_weight("kernel", (self.units, fin), init, pad=(_r8(self.units), _r8(fin)))
        self.kernel.to_keras = lambda a: a.T.copy()
        self.kernel.from_keras = lambda a: a.T.copy()
        self.bias = self.add_weight("bias", (self.units,), P.zeros, pad=(_r8(self.units),)) if self.use_bias else None

    def compute_output_shape(self, s):
        return (*s[:-1], self.units)

    def call(self, x, training=False, skip_activation=False, relu=False):
        act = self.activation_name
        fused = (act == "relu" and not skip_activation) or relu
        y = linear_ops.linear(x, self.kernel.data, None if self.bias is None else self.bias.master,
                              relu=fused, grad_w=self.kernel.grad if self.trainable else None,
                              grad_b=None if (self.bias is None or not self.trainable) else self.bias.grad,
                              on_grad=self.grad_hook, padded=self._padded())
        if not fused and not skip_activation:
            y = apply_activation(act, y)
        return y

    def _padded(self):
        """(kernel, bias master, kernel grad, bias grad) padded storage views when the arena pads
        this layer (``ops.linear.linear(padded=)``), else None."""
        k, b = self.kernel, self.bias
        if not k.padded and (b is None or not b.padded):
            return None
        return (k.pdata, None if b is None else b.pmaster, k.pgrad if self.trainable else None,
                None if (b is None or not self.trainable) else b.pgrad)

    def get_config(self):
        return {**super().get_config(), "units": self.units, "activation": self.activation_name,
                "use_bias": self.use_bias, "kernel_initializer": self.kernel_initializer}


class Conv2D(Layer):
    def __init__(self, filters, kernel_size, strides=(1, 1), padding="valid", activation=None, use_bias=True,
                 dilation_rate=(1, 1), kernel_initializer="glorot_uniform", data_format=None, **kw):
        super().__init__(**kw)
        if data_format not in (None, "channels_last"):
            raise ValueError("only channels_last (NHWC) is supported")
        self.filters = int(filters)
        self.kernel_size = _pair(kernel_size)
        self.strides = _pair(strides)
        self.padding = padding.lower() if isinstance(padding, str) else _pair(padding)
        self.dilation_rate = _pair(dilation_rate)
        self.activation_name = _act_name(activation)
        self.use_bias = use_bias
        self.kernel_initializer = kernel_initializer

    supports_skip = True

    def _pads(self, H, W):
        if isinstance(self.padding, tuple):
            return self.padding, None
        if self.padding == "valid":
            return (0, 0), None
        kh, kw = self.kernel_size
        dh, dw = self.dilation_rate
        sh, sw = self.strides
        outs = []
        for n, k, s, d in ((H, kh, sh, dh), (W, kw, sw, dw)):
            o = -(-n // s)
            total = max((o - 1) * s + (k - 1) * d + 1 - n, 0)
            outs.append((total // 2, total - total // 2))
        sym = all(a == b for a, b in outs)
        if sym:
            return (outs[0][0], outs[1][0]), None
        return (0, 0), (outs[1][0], outs[1][1], outs[0][0], outs[0][1])  # explicit F.pad (W then H)

    def build(self, input_shape):
        H, W, cin = input_shape
        kh, kw = self.kernel_size
        fan_in, fan_out = kh * kw * cin, kh * kw * self.filters
        init = P.he_normal(fan_in) if self.kernel_initializer == "he_normal" else P.glorot_uniform(fan_in, fan_out)
        self.kernel = self.add_weight("kernel", (self.filters, kh, kw, cin), init,
                                      pad=(_r8(self.filters), kh, kw, _r8(cin)))
        self.kernel.to_keras = lambda a: np.ascontiguousarray(a.transpose(1, 2, 3, 0))
        self.kernel.from_keras = lambda a: np.ascontiguousarray(a.transpose(3, 0, 1, 2))
        self.bias = self.add_weight("bias", (self.filters,), P.zeros, pad=(_r8(self.filters),)) if self.use_bias else None

    def compute_output_shape(self, s):
        H, W, _ = s
        (ph, pw), extra = self._pads(H, W)
        if extra:
            H, W = H + extra[2] + extra[3], W + extra[0] + extra[1]
        kh, kw = self.kernel_size
        dh, dw = self.dilation_rate
        sh, sw = self.strides
        return ((H + 2 * ph - dh * (kh - 1) - 1) // sh + 1, (W + 2 * pw - dw * (kw - 1) - 1) // sw + 1, self.filters)

    def call(self, x, training=False, skip_activation=False, relu=False, stats=None):
        (ph, pw), extra = self._pads(x.shape[1], x.shape[2])
        if extra:
            x = F.pad(x, (0, 0, *extra))
        fused = (self.activation_name == "relu" and not skip_activation) or relu
        y = conv_ops.conv2d(x, self.kernel.data, None if self.bias is None else self.bias.master,
                            stride=self.strides, padding=(ph, pw), dilation=self.dilation_rate, relu=fused,
                            grad_w=self.kernel.grad if self.trainable else None,
                            grad_b=None if (self.bias is None or not self.trainable) else self.bias.grad,
                            stats=stats, on_grad=self.grad_hook, padded=Dense._padded(self))
        if not fused and not skip_activation:
            y = apply_activation(self.activation_name, y)
        return y

    def get_config(self):
        return {**super().get_config(), "filters": self.filters, "kernel_size": list(self.kernel_size),
                "strides": list(self.strides),
                "padding": self.padding if isinstance(self.padding, str) else list(self.padding),
                "activation": self.activation_name,
                "use_bias": self.use_bias, "dilation_rate": list(self.dilation_rate),
                "kernel_initializer": self.kernel_initializer}


class MaxPooling2D(Layer):
    def __init__(self, pool_size=(2, 2), strides=None, padding="valid", **kw):
        super().__init__(**kw)
        self.pool_size = _pair(pool_size)
        self.strides = _pair(strides) if strides is not None else self.pool_size
        self.padding = padding.lower()

    def _pad(self):
        if self.padding == "same":
            return ((self.pool_size[0] - 1) // 2, (self.pool_size[1] - 1) // 2)
        return (0, 0)

    def compute_output_shape(self, s):
        H, W, C_ = s
        ph, pw = self._pad()
        return ((H + 2 * ph - self.pool_size[0]) // self.strides[0] + 1,
                (W + 2 * pw - self.pool_size[1]) // self.strides[1] + 1, C_)

    def call(self, x, training=False):
        return pool_ops.max_pool2d(x, self.pool_size, self.strides, self._pad())

    def get_config(self):
        return {**super().get_config(), "pool_size": list(self.pool_size), "strides": list(self.strides),
                "padding": self.padding}


class AveragePooling2D(MaxPooling2D):
    def call(self, x, training=False):
        return act_ops.avg_pool2d(x, self.pool_size, self.strides, self._pad())


class GlobalAveragePooling2D(Layer):
    def compute_output_shape(self, s):
        return (s[-1],)

    def call(self, x, training=False):
        return pool_ops.global_avg_pool(x)


class Flatten(Layer):
    def compute_output_shape(self, s):
        return (int(math.prod(s)),)

    def call(self, x, training=False):
        return x.reshape(x.shape[0], -1)


class Reshape(Layer):
    def __init__(self, target_shape, **kw):
        super().__init__(**kw)
        self.target_shape = tuple(int(t) for t in target_shape)

    def compute_output_shape(self, s):
        return self.target_shape

    def call(self, x, training=False):
        return x.reshape(x.shape[0], *self.target_shape)

    def get_config(self):
        return {**super().get_config(), "target_shape": list(self.target_shape)}


class Dropout(Layer):
    def __init__(self, rate, **kw):
        super().__init__(**kw)
        self.rate = float(rate)

    def call(self, x, training=False):
        # counter-hash mask seeded per call from a host counter (the backward regenerates it), so
        # a model containing an active Dropout trains eagerly, not from a replayed hipGraph
        return act_ops.dropout(x, self.rate, training)

    def get_config(self):
        return {**super().get_config(), "rate": self.rate}


class BatchNormalization(Layer):
    """Keras semantics: momentum is the running-average decay (0.99), epsilon 1e-3."""

    def __init__(self, axis=-1, momentum=0.99, epsilon=1e-3, center=True, scale=True, **kw):
        super().__init__(**kw)
        if axis not in (-1, 3):
            raise ValueError("BatchNormalization supports the channels-last axis only")
        self.momentum, self.epsilon, self.center, self.scale = float(momentum), float(epsilon), center, scale
        self.fuse_relu = False

    def build(self, s):
        c = int(s[-1])
        self.gamma = self.add_weight("gamma", (c,), P.ones) if self.scale else None
        self.beta = self.add_weight("beta", (c,), P.zeros) if self.center else None
        self.add_state("moving_mean", torch.zeros(c))
        self.add_state("moving_variance", torch.ones(c))

    def keras_weight_params(self):
        out = [p for p in (self.gamma, self.beta) if p is not None]
        return out + ["moving_mean", "moving_variance"]

    def call(self, x, training=False, resid=None, relu=False, stats=None):
        return norm_ops.batch_norm(
            x, None if self.gamma is None else self.gamma.master, None if self.beta is None else self.beta.master,
            self._states["moving_mean"], self._states["moving_variance"], training=training,
            momentum=1.0 - self.momentum, eps=self.epsilon, resid=resid, relu=relu or self.fuse_relu,
            grad_gamma=None if self.gamma is None else self.gamma.grad,
            grad_beta=None if self.beta is None else self.beta.grad, stats=stats, on_grad=self.grad_hook)

    def get_config(self):
        return {**super().get_config(), "momentum": self.momentum, "epsilon": self.epsilon, "center": self.center,
                "scale": self.scale}


class Embedding(Layer):
    def __init__(self, input_dim, output_dim, **kw):
        super().__init__(**kw)
        self.input_dim, self.output_dim = int(input_dim), int(output_dim)

    def build(self, s):
        self.embeddings = self.add_weight("embeddings", (self.input_dim, self.output_dim), P.uniform(0.05))

    def compute_output_shape(self, s):
        return (*s, self.output_dim)

    def call(self, x, training=False):
        from ..ops import embedding as E

        return E.embedding(x, self.embeddings.data, grad_w=self.embeddings.grad, on_grad=self.grad_hook)

    def get_config(self):
        return {**super().get_config(), "input_dim": self.input_dim, "output_dim": self.output_dim}


class _Recurrent(Layer):
    n_gates = 1
    cell = "rnn"

    def __init__(self, units, activation="tanh", recurrent_activation="hard_sigmoid", return_sequences=False,
                 use_bias=True, unit_forget_bias=True, **kw):
        super().__init__(**kw)
        self.units = int(units)
        self.activation = activation
        self.recurrent_activation = recurrent_activation
        self.return_sequences = return_sequences
        self.use_bias = use_bias
        self.unit_forget_bias = unit_forget_bias

    def build(self, s):
        T, fin = s
        G, H = self.n_gates, self.units
        self.kernel = self.add_weight("kernel", (fin, G * H), P.glorot_uniform(fin, G * H))
        self.recurrent_kernel = self.add_weight("recurrent_kernel", (H, G * H), self._orth_init(H, G))
        if self.use_bias:
            if self.cell == "lstm" and self.unit_forget_bias:
                def binit(shape, gen, H=H):
                    b = torch.zeros(shape)
                    b[H : 2 * H] = 1.0
                    return b
                self.bias = self.add_weight("bias", (G * H,), binit)
            else:
                self.bias = self.add_weight("bias", (G * H,), P.zeros)
        else:
            self.bias = None

    @staticmethod
    def _orth_init(H, G):
        def f(shape, gen):
            # Keras applies orthogonal to the whole [H, G*H] matrix
            return P.orthogonal(H, G * H)(shape, gen)
        return f

    def compute_output_shape(self, s):
        return (s[0], self.units) if self.return_sequences else (self.units,)

    def call(self, x, training=False):
        return rnn_ops.recurrent(
            self.cell, x, self.kernel.data, self.recurrent_kernel.data, None if self.bias is None else self.bias.data,
            grads=(self.kernel.grad, self.recurrent_kernel.grad, None if self.bias is None else self.bias.grad),
            return_sequences=self.return_sequences, activation=self.activation,
            recurrent_activation=self.recurrent_activation, on_grad=self.grad_hook)

    def get_config(self):
        return {**super().get_config(), "units": self.units, "activation": self.activation,
                "recurrent_activation": self.recurrent_activation, "return_sequences": self.return_sequences,
                "use_bias": self.use_bias}


class GRU(_Recurrent):
    """Keras 2 GRU (``reset_after=False``: one bias vector, 3*(in*H + H*H + H) params)."""
    n_gates = 3
    cell = "gru"


class LSTM(_Recurrent):
    """Keras 2 LSTM (gate order i, f, c, o; ``unit_forget_bias``)."""
    n_gates = 4
    cell = "lstm"

    def get_config(self):
        return {**super().get_config(), "unit_forget_bias": self.unit_forget_bias}


class SimpleRNN(_Recurrent):
    n_gates = 1
    cell = "rnn"
