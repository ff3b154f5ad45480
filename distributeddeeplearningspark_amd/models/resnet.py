"""ResNet-50 (v1.5: stride on the 3x3) in NHWC bf16 — the BASELINE.json headline model.

Every conv is followed by batch-norm; the pair is ONE fused unit on the GPU:
the conv's MFMA epilogue accumulates the per-channel BN statistics (no separate
stats sweep over the activation), and the BN apply sweep fuses the residual add and
the ReLU of the bottleneck.  Weights: He-normal convs, zero-init last BN gamma of
each block optional (``zero_init_residual``).
"""
from __future__ import annotations

import torch

from ..ops import norm as norm_ops
from ..ops._native import use_native
from . import params as P
from .core import Layer, Model
from .layers import BatchNormalization, Conv2D, Dense, Flatten, MaxPooling2D
from ..ops import pool as pool_ops


FUSED_BLOCKS = True  # bottlenecks as fused training nodes (ops/fused_blocks.py); tests compare with False


def _fused() -> bool:
    return FUSED_BLOCKS


class ConvBN(Layer):
    """conv(no bias) -> BN (training stats fused into the conv epilogue) -> [+resid] -> [ReLU]."""

    def __init__(self, filters, kernel_size, strides=1, relu=True, zero_gamma=False, bn_momentum=0.9, bn_eps=1e-5,
                 **kw):
        super().__init__(**kw)
        k = kernel_size
        self.conv = Conv2D(filters, k, strides=strides, padding=k // 2, use_bias=False, kernel_initializer="he_normal",
                           name=self.name + "/conv")
        self.bn = BatchNormalization(momentum=bn_momentum, epsilon=bn_eps, name=self.name + "/bn")
        self.relu = relu
        self.zero_gamma = zero_gamma

    def sublayers(self):
        return [self.conv, self.bn]

    def build(self, s):
        s2 = self.conv.ensure_built(s)
        self.bn.ensure_built(s2)
        if self.zero_gamma:
            self.bn.gamma.init = P.zeros

    def compute_output_shape(self, s):
        return self.conv.compute_output_shape(s)

    def call(self, x, training=False, resid=None, relu=None):
        relu = self.relu if relu is None else relu
        stats = None
        if training and use_native(x):
            stats = norm_ops.new_stats_workspace(self.conv.filters, x.device)
        y = self.conv.call(x, training, stats=stats)
        return self.bn.call(y, training, resid=resid, relu=relu, stats=stats)

    def get_config(self):
        return {**super().get_config(), "filters": self.conv.filters, "kernel_size": self.conv.kernel_size[0],
                "strides": self.conv.strides[0], "relu": self.relu}


class Bottleneck(Layer):
    expansion = 4

    def __init__(self, width, strides=1, downsample=False, zero_init_residual=False, **kw):
        super().__init__(**kw)
        out = width * self.expansion
        n = self.name
        self.c1 = ConvBN(width, 1, 1, relu=True, name=n + "/c1")
        self.c2 = ConvBN(width, 3, strides, relu=True, name=n + "/c2")
        self.c3 = ConvBN(out, 1, 1, relu=True, zero_gamma=zero_init_residual, name=n + "/c3")
        self.down = ConvBN(out, 1, strides, relu=False, name=n + "/down") if downsample else None
        self.width, self.strides, self.downsample = width, strides, downsample

    def sublayers(self):
        return [self.c1, self.c2, self.c3] + ([self.down] if self.down else [])

    def build(self, s):
        s1 = self.c1.ensure_built(s)
        s2 = self.c2.ensure_built(s1)
        self.c3.ensure_built(s2)
        if self.down:
            self.down.ensure_built(s)

    def compute_output_shape(self, s):
        H, W, _ = s
        st = self.strides
        return ((H - 1) // st + 1, (W - 1) // st + 1, self.width * self.expansion)

    def call(self, x, training=False):
        if training and use_native(x) and _fused():  # whole block as one hand-scheduled node (ops/fused_blocks.py)
            from ..ops.fused_blocks import bottleneck

            return bottleneck(self, x, self.c1.conv.kernel.data)
        sc = self.down.call(x, training) if self.down else x
        y = self.c1.call(x, training)
        y = self.c2.call(y, training)
        return self.c3.call(y, training, resid=sc)  # relu(bn(conv(y)) + shortcut), fused

    def get_config(self):
        return {**super().get_config(), "width": self.width, "strides": self.strides, "downsample": self.downsample}


class ResNet(Model):
    def __init__(self, blocks=(3, 4, 6, 3), num_classes=1000, input_shape=(224, 224, 3), zero_init_residual=False,
                 name=None, **kw):
        super().__init__(name=name or "resnet50", input_shape=input_shape, **kw)
        self.blocks, self.num_classes = tuple(blocks), int(num_classes)
        self.stem = ConvBN(64, 7, 2, relu=True, name=self.name + "/stem")
        self.stages = []
        inp = 64
        for si, (nb, w) in enumerate(zip(self.blocks, (64, 128, 256, 512))):
            st = 1 if si == 0 else 2
            for bi in range(nb):
                self.stages.append(Bottleneck(w, st if bi == 0 else 1, downsample=(bi == 0),
                                              zero_init_residual=zero_init_residual,
                                              name=f"{self.name}/s{si + 1}b{bi + 1}"))
        self.fc = Dense(self.num_classes, name=self.name + "/fc")
        self.zero_init_residual = zero_init_residual
        # uint8 ImageNet pixels fed through to_input (DataFrame path) get the standard normalisation
        self.input_mean, self.input_std = (123.675, 116.28, 103.53), (58.395, 57.12, 57.375)

    def sublayers(self):
        return [self.stem, *self.stages, self.fc]

    def build_model(self):
        if self.built:
            return
        s = tuple(self._input_shape_arg)
        self.input_shape = s
        s = self.stem.ensure_built(s)
        s = ((s[0] + 2 - 3) // 2 + 1, (s[1] + 2 - 3) // 2 + 1, s[2])  # maxpool 3x3 s2 p1
        for b in self.stages:
            s = b.ensure_built(s)
        self.fc.ensure_built((s[-1],))
        self.output_shape = (self.num_classes,)
        self.built = True

    def ends_with_softmax(self):
        return True

    def forward(self, x, training=False, logits=False):
        y = None
        if training and use_native(x) and _fused():
            from ..ops.fused_blocks import convbn_relu, stem_pool

            # stem conv + BN + ReLU + max pool in one node (the pool applies the BN on load)
            y = stem_pool(self.stem, x, self.stem.conv.kernel.data)
            if y is None:
                y = pool_ops.max_pool2d(convbn_relu(self.stem, x, self.stem.conv.kernel.data), 3, 2, 1)
        if y is None:
            y = pool_ops.max_pool2d(self.stem.call(x, training), 3, 2, 1)
        for b in self.stages:
            y = b.call(y, training)
        y = pool_ops.global_avg_pool(y)
        y = self.fc.call(y, training)
        if logits:
            return y
        from ..ops.act import activation

        return activation(y, "softmax")

    def summary_rows(self):
        rows = [(f"{l.name} ({type(l).__name__})", "", l.count_params()) for l in self.sublayers()]
        return rows

    def get_config(self):
        return {"name": self.name, "blocks": list(self.blocks), "num_classes": self.num_classes,
                "input_shape": list(self._input_shape_arg), "zero_init_residual": self.zero_init_residual}


def ResNet50(num_classes=1000, input_shape=(224, 224, 3), **kw):
    return ResNet((3, 4, 6, 3), num_classes, input_shape, **kw)


def ResNet101(num_classes=1000, input_shape=(224, 224, 3), **kw):
    return ResNet((3, 4, 23, 3), num_classes, input_shape, name=kw.pop("name", "resnet101"), **kw)
