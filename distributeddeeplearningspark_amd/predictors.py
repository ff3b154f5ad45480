"""dist-keras ``ModelPredictor``: batched inference that appends a ``prediction`` vector
column (reference: ``ddl_mnist_aztk.py:204,207``, ``ddl_nyiso_aztk.py:220-221``).

Partition-parallel like the reference (which maps a predict function over the RDD's
partitions on the executors): the frame's partitions are dealt in contiguous groups to
``num_workers`` executors (``parallel/launcher.py``: one process per MI355X, or CPU
executors), each rebuilds the model from its serialised ``{'model', 'weights'}`` blob, runs
the forward of its partitions (bf16 / fp32 HIP kernels on its GPU) and returns the rows; the
driver reassembles them in partition and row order.  With one worker (default on a single
GPU or CPU) the forward runs in-process.  Results are deterministic (unlike the reference's
lazily re-evaluated predictions).
"""
from __future__ import annotations

import os
from collections import OrderedDict

import numpy as np

from .sql import types as T
from .sql.column import ColumnData
from .sql.dataframe import DataFrame


class Predictor:
    def __init__(self, keras_model):
        self.model = keras_model if isinstance(keras_model, dict) else None
        self._live = keras_model if not isinstance(keras_model, dict) else None

    def _model(self, device=None):
        from .utils import deserialize_keras_model

        m = self._live if self._live is not None else deserialize_keras_model(self.model)
        if m.arena is None or (device is not None and str(m.device) != str(device)):
            m.place(device)
        return m

    def _blob(self):
        from .utils import serialize_keras_model

        blob = self.model if self.model is not None else serialize_keras_model(self._live)
        return {k: v for k, v in blob.items() if k not in ("optimizer", "loss")}

    def predict(self, dataframe):
        raise NotImplementedError


def _predict_partitions(rank, world, pg, blob, xs, batch_size):
    """Executor side: rebuild the model on this worker's device and predict each partition."""
    import torch

    from .utils import deserialize_keras_model, set_states

    m = deserialize_keras_model(blob)
    m.place(pg.device)
    if blob.get("flat") is not None:
        m.arena.set_flat(torch.from_numpy(blob["flat"]))
    if blob.get("states"):
        set_states(m, blob["states"])
    return [m.predict(x, batch_size=batch_size).astype(np.float32) for x in xs]


class ModelPredictor(Predictor):
    def __init__(self, keras_model, features_col="features", output_col="prediction", batch_size=1024, device=None,
                 num_workers=None):
        super().__init__(keras_model)
        self.features_column = features_col
        self.output_column = output_col
        self.batch_size = int(batch_size)
        self.device = device
        self.num_workers = num_workers

    def _workers(self, n_parts: int) -> int:
        if self.num_workers is not None:
            return max(1, min(int(self.num_workers), n_parts))
        env_world = int(os.environ.get("WORLD_SIZE", "1"))
        if env_world > 1:  # SPMD under torchrun: every rank predicts its share
            return env_world
        if self.device == "cpu":
            return 1
        from .parallel.launcher import _gpu_count

        return max(1, min(n_parts, _gpu_count()))

    def predict(self, dataframe: DataFrame) -> DataFrame:
        x = dataframe.column_array(self.features_column, None)
        slices = dataframe.partition_slices()
        nw = self._workers(len(slices))
        if nw <= 1:
            y = self._model(self.device).predict(x, batch_size=self.batch_size)
        else:
            from .parallel.launcher import run_workers

            # contiguous groups of partitions per worker keep the reassembly a concatenation
            groups = [slices[(r * len(slices)) // nw:((r + 1) * len(slices)) // nw] for r in range(nw)]
            blob = self._blob()
            args = [(blob, [x[s] for s in g], self.batch_size) for g in groups]
            outs = run_workers(_predict_partitions, nw, args, device=self.device)
            y = np.concatenate([p for per_rank in outs for p in per_rank]) if x.shape[0] else \
                np.zeros((0, 1), dtype=np.float32)
        y = np.asarray(y).astype(np.float64)
        y = y.reshape(y.shape[0], -1)
        cols = OrderedDict(dataframe._cols)
        cols[self.output_column] = ColumnData(y, None, T.VectorUDT())
        return dataframe._with(cols)


__all__ = ["Predictor", "ModelPredictor"]
