"""``DataFrameReader`` / ``DataFrameWriter``: CSV (header + inferSchema, the reference's
``com.databricks.spark.csv`` ingest, ``ddl_mnist_aztk.py:100-107``), Parquet, JSON.

Paths are local files or directories (``file://`` accepted).  ``wasb[s]://`` /
``abfs[s]://`` URIs of an account attached with ``utils.storage.attach_storage_container``
resolve to its local mount; other cloud URIs are rejected with a clear error (no network,
and the framework never ships storage credentials).
"""
from __future__ import annotations

import glob
import os
from collections import OrderedDict

import numpy as np

from . import types as T
from .column import ColumnData
from .dataframe import DataFrame, from_columns


def _local(path: str) -> list[str]:
    from ..utils.storage import resolve

    path = resolve(path)
    if path.startswith("file://"):
        path = path[len("file://"):]
    if "://" in path:
        raise IOError(f"remote storage URI {path!r} is not supported (local paths only)")
    if os.path.isdir(path):
        files = sorted(p for p in glob.glob(os.path.join(path, "*")) if not os.path.basename(p).startswith(("_", ".")))
        return files
    files = sorted(glob.glob(path))
    if not files:
        raise FileNotFoundError(path)
    return files


def _truthy(v) -> bool:
    return str(v).lower() in ("true", "1", "yes")


def _pandas_to_df(pdf, ctx, infer=True, num_partitions=1) -> DataFrame:
    data = OrderedDict()
    for c in pdf.columns:
        s = pdf[c]
        kind = s.dtype.kind
        if not infer:
            vals = np.array([None if (isinstance(x, float) and np.isnan(x)) else str(x) for x in s], dtype=object)
            data[c] = ColumnData(vals, None, T.StringType())
            continue
        if kind in "iu":
            v = s.to_numpy()
            t = T.IntegerType() if (v.size == 0 or (v.min() >= -(2 ** 31) and v.max() < 2 ** 31)) else T.LongType()
            data[c] = ColumnData(v.astype(t.np_dtype), None, t)
        elif kind == "f":
            v = s.to_numpy(dtype=np.float64)
            nan = np.isnan(v)
            data[c] = ColumnData(v, None if not nan.any() else ~nan, T.DoubleType())
        elif kind == "b":
            data[c] = ColumnData(s.to_numpy(dtype=bool), None, T.BooleanType())
        elif kind == "M":
            v = s.to_numpy().astype("datetime64[us]")
            data[c] = ColumnData(v, None if not np.isnat(v).any() else ~np.isnat(v), T.TimestampType())
        else:
            vals = np.empty(len(s), dtype=object)
            vals[:] = [None if (isinstance(x, float) and np.isnan(x)) else x for x in s.tolist()]
            m = np.array([x is not None for x in vals], dtype=bool)
            data[c] = ColumnData(vals, None if m.all() else m, T.StringType())
    return from_columns(data, ctx, num_partitions)


class DataFrameReader:
    def __init__(self, ctx):
        self._ctx = ctx
        self._fmt = "csv"
        self._opts = {}

    def format(self, source: str):
        s = source.lower()
        self._fmt = "csv" if ("csv" in s) else s
        return self

    def option(self, key, value):
        self._opts[key] = value
        return self

    def options(self, **kw):
        self._opts.update(kw)
        return self

    def schema(self, schema):
        self._opts["_schema"] = schema
        return self

    def load(self, path=None, format=None, **kw):  # noqa: A002 - pyspark signature
        if format:
            self.format(format)
        self._opts.update(kw)
        if self._fmt == "csv":
            return self.csv(path)
        if self._fmt == "parquet":
            return self.parquet(path)
        if self._fmt == "json":
            return self.json(path)
        raise ValueError(f"unsupported format {self._fmt!r}")

    def csv(self, path, header=None, inferSchema=None, sep=None, **kw):
        import pandas as pd

        o = dict(self._opts)
        o.update(kw)
        hdr = _truthy(header if header is not None else o.get("header", "false"))
        infer = _truthy(inferSchema if inferSchema is not None else o.get("inferSchema", "false"))
        sep = sep or o.get("sep", o.get("delimiter", ","))
        frames = [pd.read_csv(f, header=0 if hdr else None, sep=sep, dtype=None if infer else str,
                              keep_default_na=True) for f in _local(path)]
        pdf = pd.concat(frames, ignore_index=True) if len(frames) > 1 else frames[0]
        if not hdr:
            pdf.columns = [f"_c{i}" for i in range(pdf.shape[1])]
        df = _pandas_to_df(pdf, self._ctx, infer=infer, num_partitions=max(1, len(frames)))
        sch = o.get("_schema")
        if sch is not None:
            for f in sch.fields:
                if f.name in df.columns:
                    from .column import _cast_values

                    df._cols[f.name] = _cast_values(df._cols[f.name], f.dataType)
        return df

    def parquet(self, *paths):
        import pyarrow.parquet as pq

        files = [f for p in paths for f in _local(p)]
        pdf = pq.read_table(files[0] if len(files) == 1 else files).to_pandas()
        return _pandas_to_df(pdf, self._ctx)

    def json(self, path):
        import pandas as pd

        pdf = pd.concat([pd.read_json(f, lines=True) for f in _local(path)], ignore_index=True)
        return _pandas_to_df(pdf, self._ctx)


class DataFrameWriter:
    def __init__(self, df: DataFrame):
        self.df = df
        self._mode = "error"
        self._opts = {}

    def mode(self, m):
        self._mode = m
        return self

    def option(self, k, v):
        self._opts[k] = v
        return self

    def options(self, **kw):
        self._opts.update(kw)
        return self

    def _prep(self, path):
        if os.path.exists(path):
            if self._mode == "overwrite":
                import shutil

                shutil.rmtree(path) if os.path.isdir(path) else os.remove(path)
            elif self._mode in ("ignore",):
                return False
            elif self._mode != "append":
                raise IOError(f"path {path} already exists")
        os.makedirs(path, exist_ok=True)
        return True

    def csv(self, path, header=None, mode=None):
        if mode:
            self._mode = mode
        if not self._prep(path):
            return
        hdr = _truthy(header if header is not None else self._opts.get("header", "false"))
        for i, s in enumerate(self.df.partition_slices()):
            sub = self.df._select_rows(np.arange(s.start, s.stop), parts=[0, s.stop - s.start])
            sub.toPandas().to_csv(os.path.join(path, f"part-{i:05d}.csv"), index=False, header=hdr)

    def parquet(self, path, mode=None):
        if mode:
            self._mode = mode
        if not self._prep(path):
            return
        self.df.toPandas().to_parquet(os.path.join(path, "part-00000.parquet"))
