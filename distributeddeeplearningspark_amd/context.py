"""Spark entry points without a JVM: ``SparkConf``, ``SparkContext``, ``SQLContext``,
``SparkSession`` (reference bootstrap: ``ddl_mnist_aztk.py:62-95``).

The configuration keys the reference sets keep their meaning:
  ``spark.executor.instances`` x ``spark.executor.cores`` = number of data-parallel
  workers (``num_workers = num_executors * num_processes``, ``ddl_mnist_aztk.py:49-53``);
  on MI355X each worker is one process bound to one GPU.
  ``spark.master``: ``local[N]`` / ``local[*]`` run the workers as local processes;
  ``spark://host:port`` / ``yarn`` are accepted and treated as local (this runtime
  launches one process per GPU of the node; multi-node uses torchrun).
Everything else (serializer, locality wait, memory) is recorded and ignored.
"""
from __future__ import annotations

import os
import re
import threading

from .sql.dataframe import DataFrame, Row, from_columns
from .sql.readwriter import DataFrameReader


def _warm_device(device: str):
    """Initialise this process's HIP context and the native kernels on ``device`` (the one-GPU
    form of pre-started executors: the in-process replica group trains here)."""
    import torch

    from .ops._native import C

    d = torch.device(device)
    if d.type == "cuda":
        torch.cuda.set_device(d)
        torch.zeros(1, device=d).add_(1)
        C()
        torch.cuda.synchronize(d)


class SparkConf:
    def __init__(self, loadDefaults: bool = True):
        self._conf: dict[str, str] = {}
        if loadDefaults:
            for k, v in os.environ.items():
                if k.startswith("DDL_SPARK_"):
                    self._conf["spark." + k[len("DDL_SPARK_"):].lower().replace("_", ".")] = v

    def set(self, key, value):
        self._conf[str(key)] = str(value)
        return self

    def setIfMissing(self, key, value):
        self._conf.setdefault(str(key), str(value))
        return self

    def setAppName(self, v):
        return self.set("spark.app.name", v)

    def setMaster(self, v):
        return self.set("spark.master", v)

    def setAll(self, pairs):
        for k, v in pairs:
            self.set(k, v)
        return self

    def get(self, key, defaultValue=None):
        return self._conf.get(key, defaultValue)

    def getAll(self):
        return list(self._conf.items())

    def contains(self, key):
        return key in self._conf

    def toDebugString(self):
        return "\n".join(f"{k}={v}" for k, v in sorted(self._conf.items()))


class _HadoopConf:
    """Stand-in for ``sc._jsc.hadoopConfiguration()`` (the reference's blob-key attach,
    ``ddl_mnist_aztk.py:88-96``).  Values are kept in memory only and never logged."""

    def __init__(self):
        self._d = {}

    def get(self, k):
        return self._d.get(k)

    def set(self, k, v):
        self._d[k] = v


class _JSC:
    def __init__(self):
        self._hconf = _HadoopConf()

    def hadoopConfiguration(self):
        return self._hconf


class SparkContext:
    _active: "SparkContext | None" = None
    _lock = threading.Lock()

    def __init__(self, master=None, appName=None, conf: SparkConf | None = None, **kw):
        self._conf = conf or SparkConf()
        if master:
            self._conf.set("spark.master", master)
        if appName:
            self._conf.set("spark.app.name", appName)
        self._conf.setIfMissing("spark.master", "local[*]")
        self._conf.setIfMissing("spark.app.name", "ddl-amd")
        self._jsc = _JSC()
        self.log_level = "WARN"
        self._stopped = False
        with SparkContext._lock:
            SparkContext._active = self
        if str(self._conf.get("spark.ddl.prestartExecutors", "false")).lower() == "true":
            self.start_executors()

    def start_executors(self, device: str | None = None):
        """Start the executor processes now (``num_executors x num_processes`` of them, one
        per MI355X or co-located per ``DDL_WORKERS_PER_GPU``); they import torch, initialise
        HIP and join the process group in the background while the driver runs the ETL, as
        Spark executors are up before a job is submitted.  Trainers pick the pool up."""
        from .parallel.executors import get_pool
        from .parallel.launcher import backend_for, plan_devices

        from .parallel import replicas

        n = self.num_workers()
        if n <= 1 or int(os.environ.get("WORLD_SIZE", "1")) > 1:
            return None
        device = device or self._conf.get("spark.ddl.device") or os.environ.get("DDL_DEVICE", "auto")
        devices = plan_devices(n, device)
        if replicas.applies({"algorithm": "adag"}, devices):
            # co-located workers train as in-process replica groups (parallel/replicas.py): one executor
            # per GPU, or none at all on one GPU — the driver's own HIP context is warmed up instead
            groups = replicas.plan(devices)
            if len(groups) == 1:
                self._local_warm = threading.Thread(target=_warm_device, args=(devices[0],), daemon=True)
                self._local_warm.start()
                return None
            devices = [devices[g[0]] for g in groups]
        self._executors = get_pool(devices, backend_for(devices))
        return self._executors

    def awaitExecutors(self):
        """Block until the pre-started executors have joined their process group (the
        session-startup phase of a Spark application, before any job is submitted)."""
        pool = getattr(self, "_executors", None)
        if pool is not None and not pool.closed:
            pool.wait_ready()
        warm = getattr(self, "_local_warm", None)
        if warm is not None:
            warm.join()
            self._local_warm = None
        return self

    @classmethod
    def getOrCreate(cls, conf=None):
        return cls._active if cls._active is not None and not cls._active._stopped else cls(conf=conf)

    @property
    def master(self):
        return self._conf.get("spark.master")

    @property
    def appName(self):
        return self._conf.get("spark.app.name")

    def getConf(self):
        return self._conf

    @property
    def defaultParallelism(self) -> int:
        m = re.match(r"local\[(\d+|\*)\]", self.master or "")
        if m:
            return os.cpu_count() or 1 if m.group(1) == "*" else int(m.group(1))
        inst = int(self._conf.get("spark.executor.instances", "1"))
        cores = int(self._conf.get("spark.executor.cores", "1"))
        return inst * cores

    def num_workers(self) -> int:
        """num_executors * num_processes as the reference computes it."""
        inst = self._conf.get("spark.executor.instances")
        cores = self._conf.get("spark.executor.cores")
        if inst is not None or cores is not None:
            return int(inst or 1) * int(cores or 1)
        return self.defaultParallelism

    def setLogLevel(self, level):
        self.log_level = str(level).upper()

    def parallelize(self, data, numSlices=None):
        from .rdd import RDD

        data = list(data)
        n = numSlices or self.defaultParallelism
        n = max(1, min(n, max(len(data), 1)))
        return RDD([data[(i * len(data)) // n:((i + 1) * len(data)) // n] for i in range(n)], self)

    def stop(self):
        from .parallel.executors import shutdown_all

        self._stopped = True
        shutdown_all()  # stopping the context stops its executors (as in Spark)
        with SparkContext._lock:
            if SparkContext._active is self:
                SparkContext._active = None


class SQLContext:
    def __init__(self, sparkContext: SparkContext, sparkSession=None):
        self._sc = sparkContext
        self.sparkSession = sparkSession

    @property
    def read(self):
        return DataFrameReader(self)

    def createDataFrame(self, data, schema=None, numPartitions=None):
        return _create_df(self, data, schema, numPartitions)


def _create_df(ctx, data, schema=None, numPartitions=None):
    from collections import OrderedDict

    import numpy as np

    from .sql import types as T

    nparts = numPartitions or 1
    try:
        import pandas as pd

        if isinstance(data, pd.DataFrame):
            from .sql.readwriter import _pandas_to_df

            return _pandas_to_df(data, ctx, num_partitions=nparts)
    except ImportError:  # pragma: no cover
        pass
    if isinstance(data, dict):
        return from_columns(OrderedDict(data), ctx, nparts)
    rows = list(data)
    names = None
    stype = None
    if isinstance(schema, T.StructType):
        names, stype = schema.names, schema
    elif isinstance(schema, (list, tuple)):
        names = list(schema)
    if rows and isinstance(rows[0], dict):
        names = names or list(rows[0].keys())
        rows = [[r.get(k) for k in names] for r in rows]
    elif rows and isinstance(rows[0], Row) and rows[0].__fields__:
        names = names or list(rows[0].__fields__)
    elif rows and not isinstance(rows[0], (list, tuple)):
        rows = [[r] for r in rows]
    width = len(rows[0]) if rows else len(names or [])
    names = names or [f"_{i + 1}" for i in range(width)]
    cols = OrderedDict((n, [r[i] for r in rows]) for i, n in enumerate(names))
    return from_columns(cols, ctx, nparts, schema=stype)


class _Builder:
    def __init__(self):
        self._conf = SparkConf()

    def master(self, m):
        self._conf.set("spark.master", m)
        return self

    def appName(self, n):
        self._conf.set("spark.app.name", n)
        return self

    def config(self, key=None, value=None, conf: SparkConf | None = None):
        if conf is not None:
            for k, v in conf.getAll():
                self._conf.set(k, v)
        elif key is not None:
            self._conf.set(key, value)
        return self

    def enableHiveSupport(self):
        return self

    def getOrCreate(self) -> "SparkSession":
        if SparkSession._active is not None and not SparkSession._active.sparkContext._stopped:
            return SparkSession._active
        sc = SparkContext._active if (SparkContext._active and not SparkContext._active._stopped) else None
        if sc is None:
            sc = SparkContext(conf=self._conf)
        else:
            for k, v in self._conf.getAll():
                sc._conf.set(k, v)
        return SparkSession(sc)


class SparkSession:
    _active: "SparkSession | None" = None

    class _BuilderDescriptor:
        def __get__(self, obj, objtype=None):
            return _Builder()

    builder = _BuilderDescriptor()

    def __init__(self, sparkContext: SparkContext):
        self.sparkContext = sparkContext
        self._sc = sparkContext
        self._sql = SQLContext(sparkContext, self)
        SparkSession._active = self

    @property
    def conf(self):
        return self.sparkContext._conf

    @property
    def read(self):
        return DataFrameReader(self)

    def createDataFrame(self, data, schema=None, numPartitions=None):
        return _create_df(self, data, schema, numPartitions)

    def range(self, start, end=None, step=1, numPartitions=None):
        import numpy as np

        if end is None:
            start, end = 0, start
        return from_columns({"id": np.arange(start, end, step, dtype=np.int64)}, self, numPartitions or 1)

    def stop(self):
        self.sparkContext.stop()
        if SparkSession._active is self:
            SparkSession._active = None


__all__ = ["SparkConf", "SparkContext", "SQLContext", "SparkSession", "DataFrame", "Row"]
