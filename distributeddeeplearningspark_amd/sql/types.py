"""Spark SQL data types (the subset the reference's pipelines produce and print).

``ddl_nyiso_aztk.py:31,115`` uses ``TimestampType``; the DataFrame schemas the
notebook prints (``ddl_nyiso_hdi.ipynb:516,630``) contain ``double``, ``string``,
``timestamp``, ``vector`` and ``array<array<double>>`` columns.
"""
from __future__ import annotations

import datetime as _dt

import numpy as np


class DataType:
    def simpleString(self) -> str:
        return type(self).__name__.replace("Type", "").lower()

    def __eq__(self, other):
        return type(self) is type(other) and self.__dict__ == other.__dict__

    def __hash__(self):
        return hash(self.simpleString())

    def __repr__(self):
        return f"{type(self).__name__}()"

    # numpy storage dtype of a column of this type
    np_dtype = object


class NullType(DataType):
    pass


class StringType(DataType):
    pass


class BooleanType(DataType):
    np_dtype = np.bool_


class IntegerType(DataType):
    np_dtype = np.int32

    def simpleString(self):
        return "int"


class LongType(DataType):
    np_dtype = np.int64

    def simpleString(self):
        return "bigint"


class FloatType(DataType):
    np_dtype = np.float32


class DoubleType(DataType):
    np_dtype = np.float64


class TimestampType(DataType):
    np_dtype = "datetime64[us]"


class DateType(DataType):
    np_dtype = "datetime64[D]"


class ArrayType(DataType):
    def __init__(self, elementType: DataType, containsNull: bool = True):
        self.elementType = elementType
        self.containsNull = containsNull

    def simpleString(self):
        return f"array<{self.elementType.simpleString()}>"

    def __repr__(self):
        return f"ArrayType({self.elementType!r})"


class VectorUDT(DataType):
    """pyspark.ml.linalg.VectorUDT — stored column-wise as a 2-D float64 array."""

    def simpleString(self):
        return "vector"


class StructField:
    def __init__(self, name: str, dataType: DataType, nullable: bool = True):
        self.name, self.dataType, self.nullable = name, dataType, nullable

    def simpleString(self):
        return f"{self.name}:{self.dataType.simpleString()}"

    def __repr__(self):
        return f"StructField({self.name},{self.dataType!r},{self.nullable})"

    def __eq__(self, o):
        return isinstance(o, StructField) and (self.name, self.dataType, self.nullable) == (o.name, o.dataType, o.nullable)


class StructType(DataType):
    def __init__(self, fields=None):
        self.fields = list(fields or [])

    def add(self, name, dataType, nullable=True):
        self.fields.append(StructField(name, dataType, nullable))
        return self

    @property
    def names(self):
        return [f.name for f in self.fields]

    def __getitem__(self, k):
        if isinstance(k, int):
            return self.fields[k]
        for f in self.fields:
            if f.name == k:
                return f
        raise KeyError(k)

    def __iter__(self):
        return iter(self.fields)

    def __len__(self):
        return len(self.fields)

    def simpleString(self):
        return "struct<" + ",".join(f.simpleString() for f in self.fields) + ">"

    def __repr__(self):
        return f"StructType({self.fields!r})"


def nested_array_type(ndim: int) -> DataType:
    t: DataType = DoubleType()
    for _ in range(ndim):
        t = ArrayType(t)
    return t


def infer_type(values) -> DataType:
    """Infer a Spark type from a numpy column / python values."""
    if isinstance(values, np.ndarray):
        k = values.dtype.kind
        if values.ndim > 1:
            return nested_array_type(values.ndim - 1)
        if k == "b":
            return BooleanType()
        if k in "iu":
            return LongType() if values.dtype.itemsize > 4 else IntegerType()
        if k == "f":
            return DoubleType() if values.dtype.itemsize >= 8 else FloatType()
        if k == "M":
            return TimestampType()
        if k in "US":
            return StringType()
        for v in values:
            if v is not None:
                return infer_type_value(v)
        return NullType()
    return infer_type_value(values)


def infer_type_value(v) -> DataType:
    from ..ml.linalg import DenseVector, SparseVector

    if isinstance(v, (DenseVector, SparseVector)):
        return VectorUDT()
    if isinstance(v, bool):
        return BooleanType()
    if isinstance(v, (int, np.integer)):
        return LongType()
    if isinstance(v, (float, np.floating)):
        return DoubleType()
    if isinstance(v, (_dt.datetime, np.datetime64)):
        return TimestampType()
    if isinstance(v, str):
        return StringType()
    if isinstance(v, (list, tuple, np.ndarray)):
        inner = DoubleType()
        for e in v:
            if e is not None:
                inner = infer_type_value(e)
                break
        return ArrayType(inner)
    return StringType()
