"""``pyspark.ml.linalg`` vectors.  Columns of vectors are stored as 2-D float64 arrays
inside the DataFrame engine; these classes are what ``collect()`` returns per row."""
from __future__ import annotations

import numpy as np


class DenseVector:
    __slots__ = ("array",)

    def __init__(self, values):
        self.array = np.asarray(values, dtype=np.float64).reshape(-1)

    def toArray(self) -> np.ndarray:
        return self.array

    @property
    def values(self):
        return self.array

    def __len__(self):
        return self.array.shape[0]

    def __getitem__(self, i):
        return self.array[i]

    def __iter__(self):
        return iter(self.array.tolist())

    def __eq__(self, other):
        if isinstance(other, (DenseVector, SparseVector)):
            return np.array_equal(self.toArray(), other.toArray())
        return False

    def __array__(self, dtype=None, copy=None):
        return self.array if dtype is None else self.array.astype(dtype)

    def dot(self, other):
        return float(np.dot(self.array, np.asarray(other)))

    def norm(self, p=2):
        return float(np.linalg.norm(self.array, p))

    def __repr__(self):
        return "DenseVector([" + ", ".join(f"{v:g}" for v in self.array) + "])"

    def __str__(self):
        return "[" + ",".join(repr(float(v)) for v in self.array) + "]"


class SparseVector:
    __slots__ = ("size", "indices", "values")

    def __init__(self, size, indices, values=None):
        self.size = int(size)
        if values is None and isinstance(indices, dict):
            items = sorted(indices.items())
            indices = [k for k, _ in items]
            values = [v for _, v in items]
        self.indices = np.asarray(indices, dtype=np.int64)
        self.values = np.asarray(values, dtype=np.float64)

    def toArray(self) -> np.ndarray:
        a = np.zeros(self.size, dtype=np.float64)
        a[self.indices] = self.values
        return a

    def __len__(self):
        return self.size

    def __getitem__(self, i):
        return self.toArray()[i]

    def __eq__(self, other):
        if isinstance(other, (DenseVector, SparseVector)):
            return np.array_equal(self.toArray(), other.toArray())
        return False

    def __array__(self, dtype=None, copy=None):
        a = self.toArray()
        return a if dtype is None else a.astype(dtype)

    def __repr__(self):
        return f"SparseVector({self.size}, {dict(zip(self.indices.tolist(), self.values.tolist()))})"

    def __str__(self):
        return f"({self.size},{self.indices.tolist()},{self.values.tolist()})"


class Vectors:
    @staticmethod
    def dense(*values):
        if len(values) == 1 and not isinstance(values[0], (int, float)):
            return DenseVector(values[0])
        return DenseVector(values)

    @staticmethod
    def sparse(size, *args):
        return SparseVector(size, *args)

    @staticmethod
    def zeros(size):
        return DenseVector(np.zeros(size))
