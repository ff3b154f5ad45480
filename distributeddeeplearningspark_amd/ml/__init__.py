"""``pyspark.ml`` subset (feature transformers, linalg vectors, evaluators)."""
from . import evaluation, feature, linalg  # noqa: F401
