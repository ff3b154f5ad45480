"""``pyspark.ml.evaluation`` subset (``MulticlassClassificationEvaluator`` is imported by
the reference, ``ddl_mnist_aztk.py:41``)."""
from __future__ import annotations

import numpy as np


class MulticlassClassificationEvaluator:
    def __init__(self, predictionCol="prediction", labelCol="label", metricName="f1"):
        self.predictionCol, self.labelCol, self.metricName = predictionCol, labelCol, metricName

    def evaluate(self, df) -> float:
        p = df.column_array(self.predictionCol, np.float64).reshape(-1)
        y = df.column_array(self.labelCol, np.float64).reshape(-1)
        if self.metricName == "accuracy":
            return float((p == y).mean()) if len(y) else 0.0
        classes = np.unique(np.concatenate([p, y]))
        f1s, w = [], []
        for c in classes:
            tp = np.sum((p == c) & (y == c))
            fp = np.sum((p == c) & (y != c))
            fn = np.sum((p != c) & (y == c))
            prec = tp / (tp + fp) if tp + fp else 0.0
            rec = tp / (tp + fn) if tp + fn else 0.0
            f1s.append(2 * prec * rec / (prec + rec) if prec + rec else 0.0)
            w.append(np.sum(y == c))
        if self.metricName in ("weightedPrecision", "weightedRecall"):
            raise NotImplementedError(self.metricName)
        return float(np.average(f1s, weights=w)) if len(y) else 0.0


class RegressionEvaluator:
    def __init__(self, predictionCol="prediction", labelCol="label", metricName="rmse"):
        self.predictionCol, self.labelCol, self.metricName = predictionCol, labelCol, metricName

    def evaluate(self, df) -> float:
        p = df.column_array(self.predictionCol, np.float64).reshape(-1)
        y = df.column_array(self.labelCol, np.float64).reshape(-1)
        e = p - y
        if self.metricName == "rmse":
            return float(np.sqrt(np.mean(e ** 2)))
        if self.metricName == "mse":
            return float(np.mean(e ** 2))
        if self.metricName == "mae":
            return float(np.mean(np.abs(e)))
        if self.metricName == "r2":
            return float(1 - np.sum(e ** 2) / np.sum((y - y.mean()) ** 2))
        raise ValueError(self.metricName)
