"""``pyspark.ml.feature`` subset: ``VectorAssembler`` (used: ``ddl_mnist_aztk.py:118``,
``ddl_nyiso_aztk.py:153-170``) and the estimators the reference imports
(``OneHotEncoder``, ``StandardScaler``, ``StringIndexer``, ``ddl_mnist_aztk.py:37-41``).
All column math is vectorised numpy over the columnar store."""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

from ..sql import types as T
from ..sql.column import ColumnData
from ..sql.dataframe import DataFrame, _nonnull


def _numeric_block(cd: ColumnData) -> np.ndarray:
    v = cd.values
    if v.dtype == object:
        v = np.stack([np.asarray(x.toArray() if hasattr(x, "toArray") else x, dtype=np.float64).reshape(-1)
                      for x in v])
    v = v.astype(np.float64)
    return v.reshape(v.shape[0], -1)


class Transformer:
    def transform(self, df: DataFrame) -> DataFrame:
        raise NotImplementedError


class VectorAssembler(Transformer):
    def __init__(self, inputCols=None, outputCol=None, handleInvalid="error"):
        self.inputCols = list(inputCols or [])
        self.outputCol = outputCol or "features"
        self.handleInvalid = handleInvalid

    def setInputCols(self, v):
        self.inputCols = list(v)
        return self

    def setOutputCol(self, v):
        self.outputCol = v
        return self

    def transform(self, df: DataFrame) -> DataFrame:
        t = df._table()
        cds = [t.column(c) for c in self.inputCols]
        blocks = [_numeric_block(c) for c in cds]
        mat = np.concatenate(blocks, axis=1) if blocks else np.zeros((df._n, 0))
        ok = np.ones(df._n, dtype=bool)
        for c in cds:
            ok &= _nonnull(c) if c.values.ndim == 1 else c.valid()
        if not ok.all():
            if self.handleInvalid == "skip":
                df = df._select_rows(np.nonzero(ok)[0])
                mat = mat[ok]
            elif self.handleInvalid == "error":
                raise ValueError("VectorAssembler: null values in input columns (handleInvalid='error')")
        cols = OrderedDict(df._cols)
        cols[self.outputCol] = ColumnData(np.ascontiguousarray(mat), None, T.VectorUDT())
        return df._with(cols)


class StringIndexer:
    def __init__(self, inputCol=None, outputCol=None, handleInvalid="error"):
        self.inputCol, self.outputCol = inputCol, outputCol

    def fit(self, df):
        v = df._table().column(self.inputCol).values
        uniq, counts = np.unique(np.asarray([str(x) for x in v]), return_counts=True)
        order = np.lexsort((uniq, -counts))  # frequency desc, then alphabetical (Spark default)
        return StringIndexerModel(self.inputCol, self.outputCol, [uniq[i] for i in order])


class StringIndexerModel(Transformer):
    def __init__(self, inputCol, outputCol, labels):
        self.inputCol, self.outputCol, self.labels = inputCol, outputCol, list(labels)

    def transform(self, df):
        m = {l: i for i, l in enumerate(self.labels)}
        v = df._table().column(self.inputCol).values
        out = np.array([float(m[str(x)]) for x in v], dtype=np.float64)
        cols = OrderedDict(df._cols)
        cols[self.outputCol] = ColumnData(out, None, T.DoubleType())
        return df._with(cols)


class OneHotEncoder(Transformer):
    """Spark 2.x OneHotEncoder (dropLast=True by default) producing a vector column."""

    def __init__(self, inputCol=None, outputCol=None, dropLast=True, size=None):
        self.inputCol, self.outputCol, self.dropLast, self.size = inputCol, outputCol, dropLast, size

    def transform(self, df):
        v = df._table().column(self.inputCol).values.astype(np.int64)
        n = self.size or (int(v.max()) + 1 if len(v) else 0)
        width = n - 1 if self.dropLast else n
        out = np.zeros((len(v), width), dtype=np.float64)
        ok = v < width
        out[np.nonzero(ok)[0], v[ok]] = 1.0
        cols = OrderedDict(df._cols)
        cols[self.outputCol] = ColumnData(out, None, T.VectorUDT())
        return df._with(cols)


class StandardScaler:
    def __init__(self, inputCol=None, outputCol=None, withMean=False, withStd=True):
        self.inputCol, self.outputCol, self.withMean, self.withStd = inputCol, outputCol, withMean, withStd

    def fit(self, df):
        x = _numeric_block(df._table().column(self.inputCol))
        return StandardScalerModel(self, x.mean(0), x.std(0, ddof=1) if len(x) > 1 else np.ones(x.shape[1]))


class StandardScalerModel(Transformer):
    def __init__(self, est, mean, std):
        self.est, self.mean, self.std = est, mean, std

    def transform(self, df):
        x = _numeric_block(df._table().column(self.est.inputCol))
        if self.est.withMean:
            x = x - self.mean
        if self.est.withStd:
            x = x / np.where(self.std == 0, 1.0, self.std)
        cols = OrderedDict(df._cols)
        cols[self.est.outputCol] = ColumnData(x, None, T.VectorUDT())
        return df._with(cols)


class MinMaxScaler:
    def __init__(self, inputCol=None, outputCol=None, min=0.0, max=1.0):  # noqa: A002
        self.inputCol, self.outputCol, self.lo, self.hi = inputCol, outputCol, min, max

    def fit(self, df):
        x = _numeric_block(df._table().column(self.inputCol))
        return _MinMaxScalerModel(self, x.min(0), x.max(0))


class _MinMaxScalerModel(Transformer):
    def __init__(self, est, omin, omax):
        self.est, self.omin, self.omax = est, omin, omax

    def transform(self, df):
        x = _numeric_block(df._table().column(self.est.inputCol))
        rng = np.where(self.omax - self.omin == 0, 1.0, self.omax - self.omin)
        y = (x - self.omin) / rng * (self.est.hi - self.est.lo) + self.est.lo
        cols = OrderedDict(df._cols)
        cols[self.est.outputCol] = ColumnData(y, None, T.VectorUDT())
        return df._with(cols)
