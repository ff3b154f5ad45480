"""``pyspark.sql.functions`` subset: col/lit/udf, aggregates, lag/lead/row_number.

Reference usage: ``F.udf(lambda x: ..., TimestampType())``, ``F.col``, ``F.min``,
``F.max``, ``F.lag(col, count=n).over(w)``, ``F.lead(...)`` (``ddl_nyiso_aztk.py:115-146``).
"""
from __future__ import annotations

import builtins

import numpy as np

from . import types as T
from .column import Column, ColumnData, _Agg, _as_column, _Lit, _UDF, _Unary, _WindowFn


def col(name: str) -> Column:
    return _as_column(name)


column = col


def lit(v) -> Column:
    return Column(_Lit(v))


def udf(f=None, returnType=T.StringType()):
    """``F.udf(f, returnType)`` or decorator form.  Runs row-wise (as Python UDFs do in Spark)."""
    if isinstance(returnType, str):
        returnType = {"double": T.DoubleType(), "string": T.StringType(), "int": T.IntegerType(),
                      "timestamp": T.TimestampType()}[returnType]

    def wrap(fn):
        def call(*cols):
            return Column(_UDF(fn, returnType, [_as_column(c)._expr for c in cols]))

        call.__name__ = getattr(fn, "__name__", "udf")
        call.func = fn
        call.returnType = returnType
        return call

    if f is None:
        return wrap
    if isinstance(f, T.DataType):
        returnType = f
        return wrap
    return wrap(f)


# ------------------------------------------------------------------------------ aggregates
def _valid_vals(c: ColumnData):
    v = c.values
    if c.mask is not None:
        v = v[c.mask]
    if v.dtype.kind == "f":
        v = v[~np.isnan(v)]
    return v


def _agg(name, reducer, rtype=None):
    def f(c):
        ce = _as_column(c)._expr

        def run(cd, table):
            v = _valid_vals(cd)
            if len(v) == 0:
                return ColumnData(np.array([np.nan]), np.array([False]), rtype or cd.dtype)
            out = reducer(v)
            arr = np.array([out], dtype=v.dtype if rtype is None else rtype.np_dtype)
            return ColumnData(arr, None, rtype or cd.dtype)

        return Column(_Agg(run, ce, f"{name}({ce.name})"))

    f.__name__ = name
    return f


min = _agg("min", np.min)  # noqa: A001 - pyspark names
max = _agg("max", np.max)  # noqa: A001
sum = _agg("sum", np.sum)  # noqa: A001
avg = _agg("avg", lambda v: float(np.mean(v.astype(np.float64))), T.DoubleType())
mean = avg
stddev = _agg("stddev", lambda v: float(np.std(v.astype(np.float64), ddof=1)) if len(v) > 1 else float("nan"),
              T.DoubleType())
variance = _agg("variance", lambda v: float(np.var(v.astype(np.float64), ddof=1)) if len(v) > 1 else float("nan"),
                T.DoubleType())


def count(c="*") -> Column:
    if isinstance(c, str) and c == "*":
        return Column(_Agg(lambda cd, table: ColumnData(np.array([table.nrows], dtype=np.int64), None, T.LongType()),
                           None, "count(1)"))
    ce = _as_column(c)._expr
    return Column(_Agg(lambda cd, table: ColumnData(np.array([int(cd.valid().sum())], dtype=np.int64), None,
                                                    T.LongType()), ce, f"count({ce.name})"))


def countDistinct(c) -> Column:
    ce = _as_column(c)._expr
    return Column(_Agg(lambda cd, table: ColumnData(np.array([len(set(_valid_vals(cd).tolist()))]), None,
                                                    T.LongType()), ce, f"count(DISTINCT {ce.name})"))


# ------------------------------------------------------------------------------ window functions
def lag(c, count: int = 1, default=None, offset=None) -> Column:  # noqa: A002 - pyspark signature
    n = offset if offset is not None else count
    return Column(_WindowFn("lag", _as_column(c)._expr, int(n), default))


def lead(c, count: int = 1, default=None, offset=None) -> Column:  # noqa: A002
    n = offset if offset is not None else count
    return Column(_WindowFn("lead", _as_column(c)._expr, int(n), default))


def row_number() -> Column:
    return Column(_WindowFn("row_number", None))


def rank() -> Column:
    return Column(_WindowFn("rank", None))


# ------------------------------------------------------------------------------ scalar helpers
def _unary(name, fn, rtype=T.DoubleType()):
    def f(c):
        ce = _as_column(c)._expr
        return Column(_Unary(lambda cd: ColumnData(fn(cd.values.astype(np.float64)), cd.mask, rtype), ce,
                             f"{name}({ce.name})"))

    f.__name__ = name
    return f


abs = _unary("abs", np.abs)  # noqa: A001
sqrt = _unary("sqrt", np.sqrt)
exp = _unary("exp", np.exp)
log = _unary("log", np.log)


def when(cond: Column, value):
    return _When([(cond, value)])


class _When(Column):
    def __init__(self, branches, otherwise_v=None):
        self.branches, self.other = branches, otherwise_v
        conds = [(_as_column(c)._expr, _as_column(v)._expr) for c, v in branches]
        other = _as_column(otherwise_v)._expr if otherwise_v is not None else None

        class _E(_Unary):
            pass

        def ev(table):
            n = table.nrows
            out = other.eval(table) if other is not None else None
            vals = out.values.copy() if out is not None else np.full(n, np.nan)
            valid = out.valid().copy() if out is not None else np.zeros(n, dtype=bool)
            dtype = out.dtype if out is not None else None
            for ce, ve in reversed(conds):
                c = ce.eval(table)
                v = ve.eval(table)
                m = c.values.astype(bool) & c.valid()
                if vals.dtype != v.values.dtype:
                    vals = vals.astype(np.result_type(vals.dtype, v.values.dtype))
                vals[m] = v.values[m]
                valid[m] = v.valid()[m]
                dtype = dtype or v.dtype
            return ColumnData(vals, None if valid.all() else valid, dtype)

        class _WhenExpr(_Lit):
            pass

        e = _WhenExpr(None)
        e.name = "CASE WHEN"
        e.eval = ev
        super().__init__(e)

    def when(self, cond, value):
        return _When(self.branches + [(cond, value)], self.other)

    def otherwise(self, value):
        return _When(self.branches, value)


def monotonically_increasing_id() -> Column:
    e = _Lit(0)
    e.name = "monotonically_increasing_id()"
    e.eval = lambda table: ColumnData(np.arange(table.nrows, dtype=np.int64), None, T.LongType())
    return Column(e)


def array(*cols) -> Column:
    ces = [_as_column(c)._expr for c in cols]
    e = _Lit(0)
    e.name = f"array({', '.join(c.name for c in ces)})"

    def ev(table):
        parts = [c.eval(table) for c in ces]
        return ColumnData(np.stack([p.values.astype(np.float64) for p in parts], 1), None, T.ArrayType(T.DoubleType()))

    e.eval = ev
    return Column(e)


__all__ = ["col", "column", "lit", "udf", "min", "max", "sum", "avg", "mean", "stddev", "variance", "count",
           "countDistinct", "lag", "lead", "row_number", "rank", "abs", "sqrt", "exp", "log", "when",
           "monotonically_increasing_id", "array"]
_ = builtins
