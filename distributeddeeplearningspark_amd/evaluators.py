"""dist-keras evaluators (``AccuracyEvaluator``, ``ddl_mnist_aztk.py:203,209``) and the
reference's driver-side MAPE (``get_MAPE``, ``ddl_nyiso_aztk.py:234-242``)."""
from __future__ import annotations

import numpy as np

from .sql.dataframe import DataFrame


class Evaluator:
    def __init__(self, label_col="label", prediction_col="prediction"):
        self.label_column = label_col
        self.prediction_column = prediction_col

    def evaluate(self, dataframe: DataFrame) -> float:
        raise NotImplementedError


class AccuracyEvaluator(Evaluator):
    """Fraction of rows whose ``prediction_col`` equals ``label_col``."""

    def __init__(self, prediction_col="prediction_index", label_col="label"):
        super().__init__(label_col, prediction_col)

    def evaluate(self, dataframe):
        p = dataframe.column_array(self.prediction_column, np.float64).reshape(-1)
        y = dataframe.column_array(self.label_column, np.float64).reshape(-1)
        if len(y) == 0:
            return 0.0
        return float(np.mean(p == y))


class MAPEEvaluator(Evaluator):
    """Mean absolute percentage error in %, inf -> nan (reference semantics)."""

    def evaluate(self, dataframe):
        a = dataframe.column_array(self.label_column, np.float64)
        p = dataframe.column_array(self.prediction_column, np.float64)
        return get_MAPE(a, p)


class MSEEvaluator(Evaluator):
    def evaluate(self, dataframe):
        a = dataframe.column_array(self.label_column, np.float64).reshape(-1)
        p = dataframe.column_array(self.prediction_column, np.float64).reshape(-1)
        return float(np.mean((a - p) ** 2))


def get_MAPE(actual, pred) -> float:
    """``mean(|(a - p) / a|) * 100`` with ``inf -> nan`` exactly as ``ddl_nyiso_aztk.py:234-242``."""
    actual, pred = np.array(actual, dtype=np.float64), np.array(pred, dtype=np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        mape = np.mean(np.abs((actual - pred) / actual)) * 100
    if mape == np.inf:
        mape = np.nan
    return float(mape)


__all__ = ["Evaluator", "AccuracyEvaluator", "MAPEEvaluator", "MSEEvaluator", "get_MAPE"]
