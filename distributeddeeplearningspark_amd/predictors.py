"""dist-keras ``ModelPredictor``: batched inference that appends a ``prediction`` vector
column (reference: ``ddl_mnist_aztk.py:204,207``, ``ddl_nyiso_aztk.py:220-221``).

The features of every partition are stacked into one device-resident batch stream
and run through the model's forward on the local MI355X (bf16 kernels) or the CPU;
row order and partitioning of the input frame are preserved, so the result is
deterministic (unlike the reference's lazily re-evaluated predictions).
"""
from __future__ import annotations

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

    def predict(self, dataframe):
        raise NotImplementedError


class ModelPredictor(Predictor):
    def __init__(self, keras_model, features_col="features", output_col="prediction", batch_size=1024, device=None):
        super().__init__(keras_model)
        self.features_column = features_col
        self.output_column = output_col
        self.batch_size = int(batch_size)
        self.device = device

    def predict(self, dataframe: DataFrame) -> DataFrame:
        m = self._model(self.device)
        x = dataframe.column_array(self.features_column, np.float32)
        y = m.predict(x, batch_size=self.batch_size).astype(np.float64)
        y = y.reshape(y.shape[0], -1)
        cols = OrderedDict(dataframe._cols)
        cols[self.output_column] = ColumnData(y, None, T.VectorUDT())
        return dataframe._with(cols)


__all__ = ["Predictor", "ModelPredictor"]
