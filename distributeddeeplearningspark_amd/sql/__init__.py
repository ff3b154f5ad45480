"""``pyspark.sql`` subset: DataFrame engine, Column expressions, functions, Window, types."""
from .column import Column  # noqa: F401
from .dataframe import DataFrame, Row  # noqa: F401
from . import functions, types, window  # noqa: F401
from .window import Window  # noqa: F401
