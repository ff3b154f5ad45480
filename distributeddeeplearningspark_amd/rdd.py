"""Minimal ``pyspark.RDD`` (in-process, partitioned lists) — enough for the reference's
``df.rdd.map(lambda x: list(x[0])).collect()`` (``ddl_nyiso_aztk.py:244-245``),
``mapPartitionsWithIndex`` (the dist-keras worker entry point) and ``treeAggregate``.
Partitions are evaluated eagerly in the driver; distributed *training* never goes
through this class — it ships numpy shards to one process per GPU instead.
"""
from __future__ import annotations

import functools
import itertools
import random


class RDD:
    def __init__(self, partitions, ctx=None):
        self._parts = [list(p) for p in partitions]
        self.ctx = ctx
        self._cached = False

    # ---------------------------------------------------------------- structure
    def getNumPartitions(self) -> int:
        return len(self._parts)

    def glom(self) -> "RDD":
        return RDD([[list(p)] for p in self._parts], self.ctx)

    def cache(self):
        self._cached = True
        return self

    persist = cache

    def unpersist(self):
        self._cached = False
        return self

    def repartition(self, n: int) -> "RDD":
        flat = list(itertools.chain.from_iterable(self._parts))
        return RDD([flat[i::n] for i in range(n)], self.ctx)

    def coalesce(self, n: int, shuffle: bool = False) -> "RDD":
        if shuffle:
            return self.repartition(n)
        n = max(1, min(n, len(self._parts)))
        k = len(self._parts)
        groups = [self._parts[i * k // n:(i + 1) * k // n] for i in range(n)]
        return RDD([list(itertools.chain.from_iterable(g)) for g in groups], self.ctx)

    # ---------------------------------------------------------------- transformations
    def map(self, f) -> "RDD":
        return RDD([[f(x) for x in p] for p in self._parts], self.ctx)

    def flatMap(self, f) -> "RDD":
        return RDD([[y for x in p for y in f(x)] for p in self._parts], self.ctx)

    def filter(self, f) -> "RDD":
        return RDD([[x for x in p if f(x)] for p in self._parts], self.ctx)

    def mapPartitions(self, f, preservesPartitioning=False) -> "RDD":
        return RDD([list(f(iter(p))) for p in self._parts], self.ctx)

    def mapPartitionsWithIndex(self, f, preservesPartitioning=False) -> "RDD":
        return RDD([list(f(i, iter(p))) for i, p in enumerate(self._parts)], self.ctx)

    def zipWithIndex(self) -> "RDD":
        out, k = [], 0
        for p in self._parts:
            out.append([(x, k + i) for i, x in enumerate(p)])
            k += len(p)
        return RDD(out, self.ctx)

    def keys(self):
        return self.map(lambda kv: kv[0])

    def values(self):
        return self.map(lambda kv: kv[1])

    def reduceByKey(self, f, numPartitions=None) -> "RDD":
        acc = {}
        for p in self._parts:
            for k, v in p:
                acc[k] = f(acc[k], v) if k in acc else v
        n = numPartitions or len(self._parts)
        items = list(acc.items())
        return RDD([items[i::n] for i in range(n)], self.ctx)

    def union(self, other: "RDD") -> "RDD":
        return RDD(self._parts + other._parts, self.ctx)

    def sample(self, withReplacement, fraction, seed=None) -> "RDD":
        r = random.Random(seed)
        return RDD([[x for x in p if r.random() < fraction] for p in self._parts], self.ctx)

    # ---------------------------------------------------------------- actions
    def collect(self) -> list:
        return list(itertools.chain.from_iterable(self._parts))

    def count(self) -> int:
        return sum(len(p) for p in self._parts)

    def take(self, n: int) -> list:
        return self.collect()[:n]

    def first(self):
        for p in self._parts:
            if p:
                return p[0]
        raise ValueError("RDD is empty")

    def foreach(self, f):
        for p in self._parts:
            for x in p:
                f(x)

    def foreachPartition(self, f):
        for p in self._parts:
            f(iter(p))

    def reduce(self, f):
        vals = [functools.reduce(f, p) for p in self._parts if p]
        if not vals:
            raise ValueError("Can not reduce() empty RDD")
        return functools.reduce(f, vals)

    def fold(self, zero, op):
        return functools.reduce(op, [functools.reduce(op, p, zero) for p in self._parts], zero)

    def aggregate(self, zeroValue, seqOp, combOp):
        import copy

        parts = [functools.reduce(seqOp, p, copy.deepcopy(zeroValue)) for p in self._parts]
        return functools.reduce(combOp, parts, copy.deepcopy(zeroValue))

    def treeAggregate(self, zeroValue, seqOp, combOp, depth: int = 2):
        """Spark's treeAggregate: per-partition seqOp, then combOp in a tree of fan-in ~ n^(1/depth)."""
        import copy

        level = [functools.reduce(seqOp, p, copy.deepcopy(zeroValue)) for p in self._parts]
        if not level:
            return zeroValue
        fan = max(2, int(round(len(level) ** (1.0 / max(depth, 1)))))
        while len(level) > 1:
            level = [functools.reduce(combOp, level[i:i + fan]) for i in range(0, len(level), fan)]
        return level[0]

    def treeReduce(self, f, depth: int = 2):
        level = [functools.reduce(f, p) for p in self._parts if p]
        fan = max(2, int(round(max(len(level), 1) ** (1.0 / max(depth, 1)))))
        while len(level) > 1:
            level = [functools.reduce(f, level[i:i + fan]) for i in range(0, len(level), fan)]
        return level[0]

    def sum(self):
        return sum(self.collect())

    def mean(self):
        c = self.collect()
        return sum(c) / len(c)

    def toDF(self, schema=None):
        from .context import SparkSession

        return SparkSession.builder.getOrCreate().createDataFrame(self.collect(), schema,
                                                                  numPartitions=self.getNumPartitions())

    def __repr__(self):
        return f"RDD[{self.getNumPartitions()} partitions]"
