"""Column expressions of the DataFrame engine (``pyspark.sql.Column`` semantics).

Columns are expression trees evaluated *vectorised* against a columnar table:
every node returns a :class:`ColumnData` (numpy values + optional validity mask +
Spark type).  Python UDFs run row-wise (as in Spark); everything else is numpy.
"""
from __future__ import annotations

import datetime as _dt
import operator

import numpy as np

from . import types as T


class ColumnData:
    __slots__ = ("values", "mask", "dtype")

    def __init__(self, values, mask=None, dtype: T.DataType | None = None):
        self.values = values
        self.mask = mask  # bool array: True = valid (not null); None = all valid
        self.dtype = dtype if dtype is not None else T.infer_type(values)

    def __len__(self):
        return len(self.values)

    def valid(self) -> np.ndarray:
        return np.ones(len(self.values), dtype=bool) if self.mask is None else self.mask

    def take(self, idx) -> "ColumnData":
        return ColumnData(self.values[idx], None if self.mask is None else self.mask[idx], self.dtype)

    @staticmethod
    def concat(parts: list["ColumnData"]) -> "ColumnData":
        if not parts:
            raise ValueError("no parts")
        vals = np.concatenate([p.values for p in parts])
        if all(p.mask is None for p in parts):
            mask = None
        else:
            mask = np.concatenate([p.valid() for p in parts])
        return ColumnData(vals, mask, parts[0].dtype)


def _as_column(c) -> "Column":
    if isinstance(c, Column):
        return c
    if isinstance(c, str):
        return Column(_ColRef(c))
    return Column(_Lit(c))


def _broadcast(value, n, dtype=None) -> ColumnData:
    if value is None:
        return ColumnData(np.full(n, np.nan), np.zeros(n, dtype=bool), T.NullType())
    t = dtype or T.infer_type_value(value)
    if isinstance(value, str) or isinstance(t, T.StringType):
        arr = np.empty(n, dtype=object)
        arr[:] = value
    elif isinstance(value, _dt.datetime):
        arr = np.full(n, np.datetime64(value, "us"))
    else:
        arr = np.full(n, value)
    return ColumnData(arr, None, t)


class _Expr:
    name = "col"

    def eval(self, table) -> ColumnData:
        raise NotImplementedError

    def is_agg(self) -> bool:
        return False

    def children(self):
        return []


class _ColRef(_Expr):
    def __init__(self, name):
        self.name = name

    def eval(self, table):
        return table.column(self.name)


class _Lit(_Expr):
    def __init__(self, v):
        self.v = v
        self.name = str(v)

    def eval(self, table):
        return _broadcast(self.v, table.nrows)


_NUMERIC_RESULT = {"+", "-", "*", "/", "%", "**"}


class _BinOp(_Expr):
    OPS = {"+": operator.add, "-": operator.sub, "*": operator.mul, "/": operator.truediv, "%": np.mod,
           "**": np.power, "==": operator.eq, "!=": operator.ne, "<": operator.lt, "<=": operator.le,
           ">": operator.gt, ">=": operator.ge, "&": np.logical_and, "|": np.logical_or}

    def __init__(self, op, l, r, swap=False):
        self.op, self.l, self.r = op, l, r
        self.swap = swap
        self.name = f"({l.name} {op} {r.name})" if not swap else f"({r.name} {op} {l.name})"

    def children(self):
        return [self.l, self.r]

    def is_agg(self):
        return self.l.is_agg() or self.r.is_agg()

    def eval(self, table):
        a, b = self.l.eval(table), self.r.eval(table)
        if self.swap:
            a, b = b, a
        av, bv = a.values, b.values
        if self.op == "/":
            with np.errstate(divide="ignore", invalid="ignore"):
                out = np.true_divide(av.astype(np.float64), bv.astype(np.float64))
            bad = ~np.isfinite(out) & np.isfinite(av.astype(np.float64))  # Spark: x/0 -> null
            mask = a.valid() & b.valid() & ~bad
            return ColumnData(out, None if mask.all() else mask, T.DoubleType())
        with np.errstate(all="ignore"):
            out = self.OPS[self.op](av, bv)
        mask = None if (a.mask is None and b.mask is None) else (a.valid() & b.valid())
        if self.op in _NUMERIC_RESULT:
            dt = T.infer_type(np.asarray(out)) if isinstance(out, np.ndarray) else T.DoubleType()
        else:
            dt = T.BooleanType()
        return ColumnData(np.asarray(out), mask, dt)


class _Unary(_Expr):
    def __init__(self, fn, child, name, dtype=None):
        self.fn, self.child, self.name, self.dtype = fn, child, name, dtype

    def children(self):
        return [self.child]

    def is_agg(self):
        return self.child.is_agg()

    def eval(self, table):
        c = self.child.eval(table)
        out = self.fn(c)
        if isinstance(out, ColumnData):
            return out
        return ColumnData(np.asarray(out), c.mask, self.dtype or T.infer_type(np.asarray(out)))


class _Alias(_Expr):
    def __init__(self, child, name):
        self.child, self.name = child, name

    def children(self):
        return [self.child]

    def is_agg(self):
        return self.child.is_agg()

    def eval(self, table):
        return self.child.eval(table)


def _cast_values(c: ColumnData, t: T.DataType) -> ColumnData:
    v = c.values
    if isinstance(t, (T.DoubleType, T.FloatType)):
        if v.dtype == object:
            out = np.array([np.nan if x is None else float(x) for x in v], dtype=t.np_dtype)
        else:
            out = v.astype(t.np_dtype)
    elif isinstance(t, (T.IntegerType, T.LongType)):
        if v.dtype == object:
            out = np.array([0 if x is None else int(float(x)) for x in v], dtype=t.np_dtype)
        else:
            out = v.astype(np.float64).astype(t.np_dtype) if v.dtype.kind == "f" else v.astype(t.np_dtype)
    elif isinstance(t, T.StringType):
        out = np.array([None if x is None else str(x) for x in v], dtype=object)
    elif isinstance(t, T.BooleanType):
        out = v.astype(bool)
    elif isinstance(t, T.TimestampType):
        out = v.astype("datetime64[us]")
    else:
        out = v
    return ColumnData(out, c.mask, t)


class _Cast(_Expr):
    def __init__(self, child, t):
        self.child, self.t = child, t
        self.name = child.name

    def children(self):
        return [self.child]

    def eval(self, table):
        return _cast_values(self.child.eval(table), self.t)


class _UDF(_Expr):
    def __init__(self, f, rtype, args):
        self.f, self.rtype, self.args = f, rtype, args
        self.name = f"{getattr(f, '__name__', 'udf')}({', '.join(a.name for a in args)})"

    def children(self):
        return list(self.args)

    def eval(self, table):
        from .dataframe import to_python

        cols = [a.eval(table) for a in self.args]
        pyvals = [[to_python(c, i) for i in range(table.nrows)] for c in cols]
        out = [self.f(*row) for row in zip(*pyvals)] if cols else [self.f() for _ in range(table.nrows)]
        return from_python(out, self.rtype)


def from_python(vals, rtype: T.DataType | None) -> ColumnData:
    """Python per-row values -> ColumnData of type rtype."""
    from ..ml.linalg import DenseVector, SparseVector

    n = len(vals)
    mask = np.array([v is not None for v in vals], dtype=bool)
    if rtype is None:
        first = next((v for v in vals if v is not None), None)
        rtype = T.infer_type_value(first) if first is not None else T.NullType()
    if isinstance(rtype, T.VectorUDT):
        dim = next((len(v) for v in vals if v is not None), 0)
        arr = np.zeros((n, dim), dtype=np.float64)
        for i, v in enumerate(vals):
            if v is not None:
                arr[i] = v.toArray() if isinstance(v, (DenseVector, SparseVector)) else np.asarray(v)
    elif isinstance(rtype, T.ArrayType):
        first = next((v for v in vals if v is not None), None)
        shp = np.asarray(first, dtype=np.float64).shape if first is not None else (0,)
        arr = np.zeros((n, *shp), dtype=np.float64)
        for i, v in enumerate(vals):
            if v is not None:
                arr[i] = np.asarray(v, dtype=np.float64)
    elif isinstance(rtype, T.TimestampType):
        arr = np.array([np.datetime64(v, "us") if v is not None else np.datetime64("NaT") for v in vals],
                       dtype="datetime64[us]")
    elif isinstance(rtype, (T.DoubleType, T.FloatType)):
        arr = np.array([np.nan if v is None else float(v) for v in vals], dtype=rtype.np_dtype)
    elif isinstance(rtype, (T.IntegerType, T.LongType)):
        arr = np.array([0 if v is None else int(v) for v in vals], dtype=rtype.np_dtype)
    elif isinstance(rtype, T.BooleanType):
        arr = np.array([bool(v) if v is not None else False for v in vals], dtype=bool)
    else:
        arr = np.empty(n, dtype=object)
        arr[:] = vals
    return ColumnData(arr, None if mask.all() else mask, rtype)


class _Agg(_Expr):
    def __init__(self, fn, child, name):
        self.fn, self.child, self.name = fn, child, name

    def is_agg(self):
        return True

    def children(self):
        return [self.child]

    def eval(self, table):
        c = self.child.eval(table) if self.child is not None else None
        return self.fn(c, table)


class _WindowFn(_Expr):
    def __init__(self, kind, child, offset=1, default=None):
        self.kind, self.child, self.offset, self.default = kind, child, offset, default
        self.name = f"{kind}({child.name if child is not None else ''}, {offset})"
        self.spec = None

    def children(self):
        return [self.child] if self.child is not None else []

    def eval(self, table):
        if self.spec is None:
            raise ValueError(f"{self.kind}() needs .over(window)")
        return self.spec._apply(self, table)


class Column:
    """``pyspark.sql.Column``-compatible expression handle."""

    def __init__(self, expr: _Expr):
        self._expr = expr

    # naming
    def alias(self, name):
        return Column(_Alias(self._expr, name))

    name = alias

    @property
    def _name(self):
        return self._expr.name

    def cast(self, t):
        if isinstance(t, str):
            t = {"double": T.DoubleType(), "float": T.FloatType(), "int": T.IntegerType(), "integer": T.IntegerType(),
                 "long": T.LongType(), "bigint": T.LongType(), "string": T.StringType(), "boolean": T.BooleanType(),
                 "timestamp": T.TimestampType()}[t.lower()]
        return Column(_Cast(self._expr, t))

    astype = cast

    def over(self, window):
        e = self._expr
        if not isinstance(e, _WindowFn):
            raise TypeError("over() applies to window functions (lag/lead/row_number/rank)")
        w = _WindowFn(e.kind, e.child, e.offset, e.default)
        w.spec = window
        return Column(w)

    def isNull(self):
        return Column(_Unary(lambda c: ColumnData(~c.valid(), None, T.BooleanType()), self._expr,
                             f"({self._expr.name} IS NULL)"))

    def isNotNull(self):
        return Column(_Unary(lambda c: ColumnData(c.valid(), None, T.BooleanType()), self._expr,
                             f"({self._expr.name} IS NOT NULL)"))

    def asc(self):
        c = Column(self._expr)
        c._ascending = True
        return c

    def desc(self):
        c = Column(self._expr)
        c._ascending = False
        return c

    def between(self, lo, hi):
        return (self >= lo) & (self <= hi)

    def isin(self, *vals):
        vals = vals[0] if len(vals) == 1 and isinstance(vals[0], (list, tuple, set)) else vals
        s = set(vals)
        return Column(_Unary(lambda c: ColumnData(np.array([v in s for v in c.values], dtype=bool), c.mask,
                                                  T.BooleanType()), self._expr, f"({self._expr.name} IN {tuple(s)})"))

    def getItem(self, i):
        return Column(_Unary(lambda c: ColumnData(c.values[:, i], c.mask, T.DoubleType()), self._expr,
                             f"{self._expr.name}[{i}]"))

    __getitem__ = getItem

    def _bin(self, op, other, swap=False):
        return Column(_BinOp(op, self._expr, _as_column(other)._expr, swap))

    def __add__(self, o): return self._bin("+", o)
    def __radd__(self, o): return self._bin("+", o, True)
    def __sub__(self, o): return self._bin("-", o)
    def __rsub__(self, o): return self._bin("-", o, True)
    def __mul__(self, o): return self._bin("*", o)
    def __rmul__(self, o): return self._bin("*", o, True)
    def __truediv__(self, o): return self._bin("/", o)
    def __rtruediv__(self, o): return self._bin("/", o, True)
    def __mod__(self, o): return self._bin("%", o)
    def __pow__(self, o): return self._bin("**", o)
    def __eq__(self, o): return self._bin("==", o)  # noqa: E704
    def __ne__(self, o): return self._bin("!=", o)
    def __lt__(self, o): return self._bin("<", o)
    def __le__(self, o): return self._bin("<=", o)
    def __gt__(self, o): return self._bin(">", o)
    def __ge__(self, o): return self._bin(">=", o)
    def __and__(self, o): return self._bin("&", o)
    def __or__(self, o): return self._bin("|", o)

    def __invert__(self):
        return Column(_Unary(lambda c: ColumnData(~c.values.astype(bool), c.mask, T.BooleanType()), self._expr,
                             f"(NOT {self._expr.name})"))

    def __neg__(self):
        return Column(_Unary(lambda c: ColumnData(-c.values, c.mask, c.dtype), self._expr, f"(- {self._expr.name})"))

    __hash__ = object.__hash__

    def __bool__(self):
        raise ValueError("Cannot convert column into bool: use '&' for 'and', '|' for 'or', '~' for 'not'")

    def __repr__(self):
        return f"Column<'{self._expr.name}'>"
