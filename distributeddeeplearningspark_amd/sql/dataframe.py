"""Columnar, partitioned DataFrame engine with ``pyspark.sql.DataFrame`` semantics.

Storage: one numpy array per column over all rows (vector columns are 2-D float64,
``array<array<double>>`` columns are N-D), a validity mask per column (Spark nulls),
and partition boundaries.  ``repartition(n)`` deals rows round-robin into ``n``
contiguous partitions; one partition is one data-parallel worker (one MI355X) when a
trainer consumes the frame (reference: ``df.repartition(num_workers)``,
``ddl_mnist_aztk.py:156``).

Evaluation is eager and deterministic (the reference's lazy re-evaluation made
``limit(24)`` pick different rows between two ``show`` calls, ``ddl_nyiso_hdi.ipynb:632``
vs ``:680``; here the same rows come back every time).
"""
from __future__ import annotations

import datetime as _dt
import random
from collections import OrderedDict

import numpy as np

from . import types as T
from .column import Column, ColumnData, _Agg, _Alias, _as_column, _ColRef, from_python


class AnalysisException(Exception):
    pass


class Row(tuple):
    """``pyspark.sql.Row``: tuple with named fields."""

    def __new__(cls, *args, **kwargs):
        if kwargs:
            names = list(kwargs)
            r = tuple.__new__(cls, [kwargs[k] for k in names])
            r.__fields__ = names
            return r
        r = tuple.__new__(cls, args)
        r.__fields__ = None
        return r

    @classmethod
    def _make(cls, names, vals):
        r = tuple.__new__(cls, vals)
        r.__fields__ = list(names)
        return r

    def asDict(self, recursive=False):
        return dict(zip(self.__fields__ or [], self))

    def __getattr__(self, item):
        f = tuple.__getattribute__(self, "__dict__").get("__fields__")
        if f and item in f:
            return self[f.index(item)]
        raise AttributeError(item)

    def __getitem__(self, k):
        if isinstance(k, str):
            return tuple.__getitem__(self, self.__fields__.index(k))
        return tuple.__getitem__(self, k)

    def __contains__(self, item):
        return item in (self.__fields__ or [])

    def __repr__(self):
        if self.__fields__:
            return "Row(" + ", ".join(f"{k}={v!r}" for k, v in zip(self.__fields__, self)) + ")"
        return "<Row(" + ", ".join(repr(v) for v in self) + ")>"

    def __reduce__(self):
        return (Row._make, (self.__fields__, tuple(self)))


def to_python(cd: ColumnData, i: int):
    from ..ml.linalg import DenseVector

    if cd.mask is not None and not cd.mask[i]:
        return None
    v = cd.values[i]
    t = cd.dtype
    if isinstance(t, T.VectorUDT):
        return DenseVector(v)
    if isinstance(t, T.ArrayType):
        return v.tolist() if isinstance(v, np.ndarray) else v
    if isinstance(t, T.TimestampType):
        if np.isnat(v):
            return None
        return v.astype("datetime64[us]").astype(_dt.datetime)
    if isinstance(v, np.generic):
        if isinstance(v, np.floating) and np.isnan(v) and isinstance(t, T.NullType):
            return None
        return v.item()
    return v


def _fmt_cell(v, truncate):
    from ..ml.linalg import DenseVector, SparseVector

    if v is None:
        s = "null"
    elif isinstance(v, (DenseVector, SparseVector)):
        s = str(v)
    elif isinstance(v, list):
        def rec(x):
            return "WrappedArray(" + ", ".join(rec(e) for e in x) + ")" if isinstance(x, list) else repr(float(x))
        s = "[" + ", ".join(rec(e) for e in v) + "]"
    elif isinstance(v, _dt.datetime):
        s = v.strftime("%Y-%m-%d %H:%M:%S")
    elif isinstance(v, float):
        s = repr(v)
    else:
        s = str(v)
    if truncate and len(s) > 20:
        s = s[:17] + "..."
    return s


class _Table:
    def __init__(self, cols: "OrderedDict[str, ColumnData]", nrows: int):
        self.cols = cols
        self.nrows = nrows

    def column(self, name: str) -> ColumnData:
        if name in self.cols:
            return self.cols[name]
        raise AnalysisException(f"cannot resolve '`{name}`' given input columns: [{', '.join(self.cols)}]")


class DataFrameNaFunctions:
    def __init__(self, df):
        self.df = df

    def drop(self, how="any", thresh=None, subset=None):
        df = self.df
        names = subset if subset is not None else df.columns
        if isinstance(names, str):
            names = [names]
        if not names or df._n == 0:
            return df
        valid = np.stack([_nonnull(df._cols[c]) for c in names], 1)
        if thresh is not None:
            keep = valid.sum(1) >= thresh
        elif how == "all":
            keep = valid.any(1)
        else:
            keep = valid.all(1)
        return df._select_rows(np.nonzero(keep)[0])

    def fill(self, value, subset=None):
        df = self.df
        names = subset if subset is not None else df.columns
        if isinstance(names, str):
            names = [names]
        cols = OrderedDict(df._cols)
        for c in names:
            cd = cols[c]
            v = value[c] if isinstance(value, dict) else value
            if isinstance(v, dict) or v is None:
                continue
            ok = _nonnull(cd)
            if ok.all():
                continue
            vals = cd.values.copy()
            try:
                vals[~ok] = v
            except (TypeError, ValueError):
                continue
            cols[c] = ColumnData(vals, None, cd.dtype)
        return df._with(cols)


def _nonnull(cd: ColumnData) -> np.ndarray:
    ok = cd.valid().copy()
    v = cd.values
    if v.dtype.kind == "f" and v.ndim == 1:
        ok &= ~np.isnan(v)
    elif v.dtype == object:
        ok &= np.array([x is not None for x in v], dtype=bool)
    elif v.dtype.kind == "M":
        ok &= ~np.isnat(v)
    return ok


class GroupedData:
    def __init__(self, df, keys):
        self.df, self.keys = df, keys

    def agg(self, *exprs):
        df = self.df
        if len(exprs) == 1 and isinstance(exprs[0], dict):
            from . import functions as F

            exprs = [getattr(F, fn)(c) for c, fn in exprs[0].items()]
        keyvals = [df._cols[k] for k in self.keys]
        groups = OrderedDict()
        for i in range(df._n):
            key = tuple(to_python(kv, i) for kv in keyvals)
            groups.setdefault(key, []).append(i)
        out_cols = OrderedDict((k, []) for k in self.keys)
        names = [(_as_column(e)._expr.name) for e in exprs]
        for n in names:
            out_cols[n] = []
        for key, idx in groups.items():
            sub = df._select_rows(np.array(idx))
            for k, v in zip(self.keys, key):
                out_cols[k].append(v)
            t = _Table(sub._cols, sub._n)
            for n, e in zip(names, exprs):
                out_cols[n].append(to_python(_as_column(e)._expr.eval(t), 0))
        cols = OrderedDict((k, from_python(v, None)) for k, v in out_cols.items())
        return DataFrame(cols, len(groups), None, df._ctx)

    def count(self):
        from . import functions as F

        return self.agg(F.count("*").alias("count"))

    def _simple(fname):
        def f(self, *cols):
            from . import functions as F

            return self.agg(*[getattr(F, fname)(c) for c in cols])
        return f

    min = _simple("min")  # noqa: A003
    max = _simple("max")  # noqa: A003
    sum = _simple("sum")  # noqa: A003
    avg = _simple("avg")
    mean = _simple("avg")


class DataFrame:
    def __init__(self, cols: "OrderedDict[str, ColumnData]", nrows: int, parts=None, ctx=None):
        self._cols = OrderedDict(cols)
        self._n = int(nrows)
        self._parts = list(parts) if parts is not None else [0, self._n]
        self._ctx = ctx
        self.is_cached = False

    # ---------------------------------------------------------------- basics
    def _with(self, cols, nrows=None, parts=None):
        n = self._n if nrows is None else nrows
        return DataFrame(cols, n, self._parts if parts is None and nrows is None else parts, self._ctx)

    @property
    def columns(self):
        return list(self._cols)

    @property
    def schema(self) -> T.StructType:
        return T.StructType([T.StructField(k, v.dtype, True) for k, v in self._cols.items()])

    @property
    def dtypes(self):
        return [(k, v.dtype.simpleString()) for k, v in self._cols.items()]

    def printSchema(self):
        print("root")
        for k, v in self._cols.items():
            print(f" |-- {k}: {v.dtype.simpleString()} (nullable = true)")

    def __getitem__(self, item):
        if isinstance(item, str):
            return _as_column(item)
        if isinstance(item, Column):
            return self.filter(item)
        if isinstance(item, (list, tuple)):
            return self.select(*item)
        raise TypeError(item)

    def __getattr__(self, item):
        if item.startswith("_"):
            raise AttributeError(item)
        if item in self._cols:
            return _as_column(item)
        raise AttributeError(item)

    def _table(self):
        return _Table(self._cols, self._n)

    def _select_rows(self, idx, parts=None):
        idx = np.asarray(idx, dtype=np.int64)
        cols = OrderedDict((k, v.take(idx)) for k, v in self._cols.items())
        if parts is None:
            # keep rows in their partitions
            pid = np.searchsorted(self._parts, idx, side="right") - 1
            counts = np.bincount(pid, minlength=len(self._parts) - 1) if len(idx) else np.zeros(
                len(self._parts) - 1, dtype=np.int64)
            parts = [0] + np.cumsum(counts).tolist()
        return DataFrame(cols, len(idx), parts, self._ctx)

    # ---------------------------------------------------------------- projection
    def _eval_named(self, c):
        if isinstance(c, str):
            if c == "*":
                return [(k, v) for k, v in self._cols.items()]
            return [(c, self._table().column(c))]
        e = _as_column(c)._expr
        return [(e.name, e.eval(self._table()))]

    def select(self, *cols):
        if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
            cols = tuple(cols[0])
        exprs = [_as_column(c) if not (isinstance(c, str) and c == "*") else c for c in cols]
        is_agg = [not isinstance(c, str) and c._expr.is_agg() for c in exprs]
        out = OrderedDict()
        if any(is_agg):
            if not all(is_agg):
                raise AnalysisException("cannot mix aggregate and non-aggregate columns without groupBy")
            t = self._table()
            for c in exprs:
                out[c._expr.name] = c._expr.eval(t)
            return DataFrame(out, 1, None, self._ctx)
        for c in exprs:
            for k, v in self._eval_named(c):
                out[k] = v
        return self._with(out)

    def selectExpr(self, *exprs):
        return self.select(*exprs)

    def withColumn(self, name, col: Column):
        cd = _as_column(col)._expr.eval(self._table())
        if len(cd) != self._n:
            raise AnalysisException("withColumn: expression produced a different number of rows")
        cols = OrderedDict(self._cols)
        cols[name] = cd
        return self._with(cols)

    def withColumnRenamed(self, old, new):
        cols = OrderedDict((new if k == old else k, v) for k, v in self._cols.items())
        return self._with(cols)

    def drop(self, *names):
        names = [n if isinstance(n, str) else n._expr.name for n in names]
        return self._with(OrderedDict((k, v) for k, v in self._cols.items() if k not in names))

    def filter(self, cond):
        if isinstance(cond, str):
            raise AnalysisException("string filter expressions are not supported; use Column expressions")
        cd = _as_column(cond)._expr.eval(self._table())
        keep = cd.values.astype(bool) & cd.valid()
        return self._select_rows(np.nonzero(keep)[0])

    where = filter

    @property
    def na(self):
        return DataFrameNaFunctions(self)

    def dropna(self, how="any", thresh=None, subset=None):
        return self.na.drop(how, thresh, subset)

    def fillna(self, value, subset=None):
        return self.na.fill(value, subset)

    # ---------------------------------------------------------------- row-order operations
    def limit(self, n: int):
        n = max(0, min(int(n), self._n))
        return self._select_rows(np.arange(n), parts=[0, n])

    def orderBy(self, *cols, ascending=True):
        if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
            cols = tuple(cols[0])
        asc = ascending if isinstance(ascending, (list, tuple)) else [ascending] * len(cols)
        from .window import _sort_keys

        cs = [_as_column(c) for c in cols]
        cds = [c._expr.eval(self._table()) for c in cs]
        keys = _sort_keys(cds)
        adj = []
        for k, c, a in zip(keys, cs, asc):
            a = getattr(c, "_ascending", a)
            kk = k.astype(np.int64) if k.dtype.kind == "M" else k
            adj.append(kk if a else -kk.astype(np.float64))
        idx = np.lexsort(list(reversed(adj))) if adj else np.arange(self._n)
        return self._select_rows(idx, parts=[0, self._n])

    sort = orderBy

    def repartition(self, numPartitions, *cols):
        n = int(numPartitions)
        if n < 1:
            raise ValueError("numPartitions must be >= 1")
        # round-robin dealing: row j -> partition j % n, each partition contiguous
        order = np.concatenate([np.arange(p, self._n, n) for p in range(n)]) if self._n else np.arange(0)
        sizes = [len(range(p, self._n, n)) for p in range(n)]
        parts = [0] + np.cumsum(sizes).tolist()
        df = self._select_rows(order, parts=parts)
        return df

    def coalesce(self, numPartitions):
        k = self.rdd_partitions_count()
        n = max(1, min(int(numPartitions), k))
        bounds = [self._parts[(i * k) // n] for i in range(n)] + [self._n]
        return DataFrame(self._cols, self._n, bounds, self._ctx)

    def rdd_partitions_count(self):
        return len(self._parts) - 1

    def partition_slices(self):
        return [slice(self._parts[i], self._parts[i + 1]) for i in range(len(self._parts) - 1)]

    def cache(self):
        self.is_cached = True
        return self

    def persist(self, *a, **k):
        return self.cache()

    def unpersist(self, *a, **k):
        self.is_cached = False
        return self

    def distinct(self):
        seen, keep = set(), []
        rows = self.collect()
        for i, r in enumerate(rows):
            key = tuple(str(v) for v in r)
            if key not in seen:
                seen.add(key)
                keep.append(i)
        return self._select_rows(np.array(keep, dtype=np.int64))

    dropDuplicates = distinct

    def union(self, other: "DataFrame"):
        if len(other.columns) != len(self.columns):
            raise AnalysisException("union: different number of columns")
        cols = OrderedDict()
        for (k, a), b in zip(self._cols.items(), other._cols.values()):
            cols[k] = ColumnData.concat([a, ColumnData(b.values.astype(a.values.dtype) if a.values.dtype != object
                                                       else b.values, b.mask, a.dtype)])
        parts = self._parts + [p + self._n for p in other._parts[1:]]
        return DataFrame(cols, self._n + other._n, parts, self._ctx)

    unionAll = union

    def randomSplit(self, weights, seed=None):
        rng = np.random.default_rng(seed)
        w = np.asarray(weights, dtype=np.float64)
        w = w / w.sum()
        u = rng.random(self._n)
        edges = np.cumsum(w)
        which = np.searchsorted(edges, u, side="right")
        return [self._select_rows(np.nonzero(which == i)[0]) for i in range(len(w))]

    def sample(self, withReplacement=False, fraction=0.1, seed=None):
        rng = np.random.default_rng(seed)
        return self._select_rows(np.nonzero(rng.random(self._n) < fraction)[0])

    def groupBy(self, *cols):
        cols = cols[0] if len(cols) == 1 and isinstance(cols[0], (list, tuple)) else cols
        return GroupedData(self, [c if isinstance(c, str) else c._expr.name for c in cols])

    groupby = groupBy

    def agg(self, *exprs):
        return self.select(*exprs)

    # ---------------------------------------------------------------- actions
    def count(self) -> int:
        return self._n

    def collect(self):
        names = self.columns
        cds = list(self._cols.values())
        return [Row._make(names, [to_python(c, i) for c in cds]) for i in range(self._n)]

    def take(self, n):
        return self.limit(n).collect()

    def head(self, n=None):
        if n is None:
            r = self.take(1)
            return r[0] if r else None
        return self.take(n)

    def first(self):
        return self.head()

    def toLocalIterator(self):
        return iter(self.collect())

    def show(self, n=20, truncate=True, vertical=False):
        print(self._show_string(n, truncate))

    def _show_string(self, n=20, truncate=True):
        rows = self.take(n)
        names = self.columns
        cells = [[_fmt_cell(v, truncate) for v in r] for r in rows]
        widths = [max([len(h)] + [len(r[i]) for r in cells] + [3]) for i, h in enumerate(names)]
        sep = "+" + "+".join("-" * w for w in widths) + "+"
        lines = [sep, "|" + "|".join(h.rjust(w) for h, w in zip(names, widths)) + "|", sep]
        for r in cells:
            lines.append("|" + "|".join(c.rjust(w) for c, w in zip(r, widths)) + "|")
        lines.append(sep)
        if self._n > n:
            lines.append(f"only showing top {n} row{'s' if n != 1 else ''}")
        return "\n".join(lines) + "\n"

    def toPandas(self):
        import pandas as pd

        data = OrderedDict()
        for k, cd in self._cols.items():
            if cd.values.ndim == 1 and cd.values.dtype != object and cd.mask is None:
                data[k] = cd.values
            else:
                data[k] = [to_python(cd, i) for i in range(self._n)]
        return pd.DataFrame(data)

    def describe(self, *cols):
        from . import functions as F

        cols = list(cols) or [k for k, v in self._cols.items() if v.values.ndim == 1 and v.values.dtype.kind in "iuf"]
        stats = OrderedDict(summary=["count", "mean", "stddev", "min", "max"])
        for c in cols:
            v = self._cols[c].values.astype(np.float64)
            v = v[_nonnull(self._cols[c])]
            stats[c] = [str(len(v)), str(v.mean() if len(v) else None), str(v.std(ddof=1) if len(v) > 1 else None),
                        str(v.min() if len(v) else None), str(v.max() if len(v) else None)]
        return DataFrame(OrderedDict((k, from_python(v, T.StringType())) for k, v in stats.items()), 5, None,
                         self._ctx)

    # ---------------------------------------------------------------- rdd / numpy bridges
    @property
    def rdd(self):
        from ..rdd import RDD

        rows = self.collect()
        return RDD([rows[s] for s in self.partition_slices()], self._ctx)

    def column_array(self, name: str, dtype=np.float32) -> np.ndarray:
        """Dense numpy view of a (vector / array / scalar) column for the trainers.

        ``dtype=None`` keeps the column's own element type (uint8 image tensors stay uint8,
        integer labels stay integers) and only narrows float64 to float32 — what the
        trainers ship to the workers, so an ImageNet-shape frame is not inflated 4x."""
        cd = self._table().column(name)
        v = cd.values
        if v.dtype == object:
            v = np.stack([np.asarray(x.toArray() if hasattr(x, "toArray") else x, dtype=np.float64) for x in v])
        if dtype is None:
            dtype = np.float32 if v.dtype.kind == "f" else (np.int64 if v.dtype.kind == "b" else v.dtype)
        return np.ascontiguousarray(v.astype(dtype, copy=False))

    def partition_arrays(self, cols, dtype=np.float32):
        """[(array per col) per partition] — how a trainer ships each shard to its worker
        (zero-copy slices of one array per column; ``dtype=None``: see :meth:`column_array`)."""
        full = [self.column_array(c, dtype) for c in cols]
        return [[a[s] for a in full] for s in self.partition_slices()]

    @property
    def write(self):
        from .readwriter import DataFrameWriter

        return DataFrameWriter(self)

    def __repr__(self):
        return "DataFrame[" + ", ".join(f"{k}: {t}" for k, t in self.dtypes) + "]"


def from_columns(data: "OrderedDict[str, object]", ctx=None, num_partitions: int = 1, schema=None) -> DataFrame:
    cols = OrderedDict()
    n = None
    for i, (k, v) in enumerate(data.items()):
        t = None
        if schema is not None:
            t = schema.fields[i].dataType
        if isinstance(v, ColumnData):
            cd = v
        elif isinstance(v, np.ndarray) and v.dtype != object:
            if v.dtype.kind == "M":
                v = v.astype("datetime64[us]")
                cd = ColumnData(v, None if not np.isnat(v).any() else ~np.isnat(v), T.TimestampType())
            else:
                cd = ColumnData(v, None, t or T.infer_type(v))
        else:
            cd = from_python(list(v), t)
        cols[k] = cd
        n = len(cd) if n is None else n
        if len(cd) != n:
            raise ValueError("columns of different length")
    n = n or 0
    k = max(1, int(num_partitions))
    parts = [(i * n) // k for i in range(k)] + [n]
    return DataFrame(cols, n, parts, ctx)
