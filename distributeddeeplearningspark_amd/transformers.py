"""dist-keras ``distkeras.transformers`` API on the columnar DataFrame engine.

Reference usage (constructor kwargs kept verbatim):
  ``MinMaxTransformer(n_min, n_max, o_min, o_max, input_col, output_col, is_vector)``
      scalar mode ``ddl_nyiso_aztk.py:123-136``, vector mode ``ddl_mnist_aztk.py:133-139``,
      inverse use (ranges swapped) ``ddl_nyiso_aztk.py:225-231``
  ``OneHotTransformer(nb_classes, input_col, output_col)``  ``ddl_mnist_aztk.py:126``
  ``ReshapeTransformer(input_col, output_col, shape)``       ``ddl_mnist_aztk.py:142``
  ``DenseTransformer(input_col, output_col)``               ``ddl_mnist_aztk.py:150``
  ``LabelIndexTransformer(output_dim)``                     ``ddl_mnist_aztk.py:205``
Every transform is one vectorised numpy pass over the column (no per-row Python), or —
with ``device="cuda"`` / ``DDL_ETL_DEVICE=cuda`` — one fp64 HIP kernel on the GPU
(``ops/etl.py``, ``csrc/kernels/ingest.hip``) with identical results.
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

from .ops import etl as E
from .sql import types as T
from .sql.column import ColumnData
from .sql.dataframe import DataFrame


def _block(df: DataFrame, col: str) -> tuple[np.ndarray, ColumnData]:
    cd = df._table().column(col)
    v = cd.values
    if v.dtype == object:
        v = np.stack([np.asarray(x.toArray() if hasattr(x, "toArray") else x, dtype=np.float64) for x in v])
    return v, cd


def _with(df: DataFrame, name: str, cd: ColumnData) -> DataFrame:
    cols = OrderedDict(df._cols)
    cols[name] = cd
    return df._with(cols)


class Transformer:
    def transform(self, dataframe: DataFrame) -> DataFrame:
        raise NotImplementedError


class MinMaxTransformer(Transformer):
    """Affine rescale [o_min, o_max] -> [n_min, n_max]; ``is_vector`` selects a vector
    (DenseVector) or scalar (double) output column."""

    def __init__(self, o_min, o_max, n_min, n_max, input_col, output_col, is_vector=True, device=None):
        self.device = device
        self.o_min, self.o_max = float(o_min), float(o_max)
        self.n_min, self.n_max = float(n_min), float(n_max)
        self.input_col, self.output_col, self.is_vector = input_col, output_col, is_vector
        rng = self.o_max - self.o_min
        self.scale = (self.n_max - self.n_min) / rng if rng != 0 else 0.0

    def transform(self, dataframe):
        v, cd = _block(dataframe, self.input_col)
        dev = E.etl_device(self.device)
        if dev is not None:
            out = E.minmax(v, self.o_min, self.scale, self.n_min, dev)
        else:
            out = (v.astype(np.float64) - self.o_min) * self.scale + self.n_min
        if self.is_vector:
            out = out.reshape(out.shape[0], -1)
            return _with(dataframe, self.output_col, ColumnData(out, cd.mask, T.VectorUDT()))
        return _with(dataframe, self.output_col, ColumnData(out.reshape(-1), cd.mask, T.DoubleType()))


class OneHotTransformer(Transformer):
    def __init__(self, output_dim, input_col, output_col, device=None):
        self.output_dim, self.input_col, self.output_col = int(output_dim), input_col, output_col
        self.device = device

    def transform(self, dataframe):
        v, cd = _block(dataframe, self.input_col)
        idx = v.reshape(-1).astype(np.int64)
        dev = E.etl_device(self.device)
        if dev is not None:
            return _with(dataframe, self.output_col, ColumnData(E.one_hot(idx, self.output_dim, dev), cd.mask,
                                                                T.VectorUDT()))
        if len(idx) and (idx.min() < 0 or idx.max() >= self.output_dim):
            raise ValueError(f"OneHotTransformer: label outside [0, {self.output_dim})")
        out = np.zeros((len(idx), self.output_dim), dtype=np.float64)
        out[np.arange(len(idx)), idx] = 1.0
        return _with(dataframe, self.output_col, ColumnData(out, cd.mask, T.VectorUDT()))


class ReshapeTransformer(Transformer):
    """Vector -> nested array of ``shape`` (schema ``array<array<...double>>``,
    ``ddl_nyiso_hdi.ipynb:516``)."""

    def __init__(self, input_col, output_col, shape):
        self.input_col, self.output_col, self.shape = input_col, output_col, tuple(int(s) for s in shape)

    def transform(self, dataframe):
        v, cd = _block(dataframe, self.input_col)
        out = v.reshape((v.shape[0],) + self.shape).astype(np.float64)
        return _with(dataframe, self.output_col, ColumnData(out, cd.mask, T.nested_array_type(len(self.shape))))


class DenseTransformer(Transformer):
    """Sparse vector column -> dense vector column (storage is already dense; this
    materialises the column under the new name with the vector type)."""

    def __init__(self, input_col, output_col):
        self.input_col, self.output_col = input_col, output_col

    def transform(self, dataframe):
        v, cd = _block(dataframe, self.input_col)
        return _with(dataframe, self.output_col,
                     ColumnData(v.reshape(v.shape[0], -1).astype(np.float64), cd.mask, T.VectorUDT()))


class LabelIndexTransformer(Transformer):
    """Prediction vector -> class index (argmax).  ``activation_threshold``: when set,
    rows whose maximum activation is below it get ``default_index``."""

    def __init__(self, output_dim, input_col="prediction", output_col="prediction_index", default_index=0,
                 activation_threshold=None, device=None):
        self.device = device
        self.output_dim, self.input_col, self.output_col = int(output_dim), input_col, output_col
        self.default_index, self.activation_threshold = default_index, activation_threshold

    def transform(self, dataframe):
        v, cd = _block(dataframe, self.input_col)
        v = v.reshape(v.shape[0], -1)[:, : self.output_dim]
        dev = E.etl_device(self.device)
        if dev is not None and len(v):
            idx = E.argmax(v, dev).astype(np.float64)
        else:
            idx = np.argmax(v, axis=1).astype(np.float64) if len(v) else np.zeros(0)
        if self.activation_threshold is not None and len(v):
            idx = np.where(v.max(1) >= self.activation_threshold, idx, float(self.default_index))
        return _with(dataframe, self.output_col, ColumnData(idx, cd.mask, T.DoubleType()))


class BinaryLabelTransformer(Transformer):
    def __init__(self, input_col, output_col, label, output_dim=2):
        self.input_col, self.output_col, self.label, self.output_dim = input_col, output_col, label, output_dim

    def transform(self, dataframe):
        v, cd = _block(dataframe, self.input_col)
        pos = (v.reshape(-1) == self.label).astype(np.int64)
        out = np.zeros((len(pos), self.output_dim))
        out[np.arange(len(pos)), pos] = 1.0
        return _with(dataframe, self.output_col, ColumnData(out, cd.mask, T.VectorUDT()))


class StandardTransformer(Transformer):
    """Column standardisation (x - mean) / std with statistics over the whole frame."""

    def __init__(self, input_col, output_col, is_vector=True):
        self.input_col, self.output_col, self.is_vector = input_col, output_col, is_vector
        self.mean = self.std = None

    def transform(self, dataframe):
        v, cd = _block(dataframe, self.input_col)
        v = v.astype(np.float64)
        if self.mean is None:
            self.mean = v.mean(0)
            self.std = np.where(v.std(0) == 0, 1.0, v.std(0))
        out = (v - self.mean) / self.std
        t = T.VectorUDT() if self.is_vector else T.DoubleType()
        return _with(dataframe, self.output_col, ColumnData(out.reshape(out.shape[0], -1) if self.is_vector
                                                            else out.reshape(-1), cd.mask, t))


__all__ = ["Transformer", "MinMaxTransformer", "OneHotTransformer", "ReshapeTransformer", "DenseTransformer",
           "LabelIndexTransformer", "BinaryLabelTransformer", "StandardTransformer"]
