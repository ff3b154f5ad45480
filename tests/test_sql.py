"""DataFrame engine vs pandas (the reference's Spark SQL surface)."""
import datetime as dt

import numpy as np
import pandas as pd
import pytest

from distributeddeeplearningspark_amd.context import SparkConf, SparkContext, SparkSession, SQLContext
from distributeddeeplearningspark_amd.ml.feature import OneHotEncoder, StandardScaler, StringIndexer, VectorAssembler
from distributeddeeplearningspark_amd.ml.linalg import DenseVector, SparseVector, Vectors
from distributeddeeplearningspark_amd.sql import Row, Window
from distributeddeeplearningspark_amd.sql import functions as F
from distributeddeeplearningspark_amd.sql.types import TimestampType


@pytest.fixture(scope="module")
def spark():
    if SparkSession._active is not None:
        SparkSession._active.stop()
    conf = SparkConf().set("spark.master", "local[2]").set("spark.executor.instances", 2).set("spark.executor.cores", 2)
    sc = SparkContext(conf=conf)
    s = SparkSession.builder.getOrCreate()
    yield s
    sc.stop()


def test_conf_and_topology(spark):
    sc = spark.sparkContext
    assert sc.num_workers() == 4  # num_executors * num_processes (ddl_mnist_aztk.py:53)
    assert sc.getConf().get("spark.master") == "local[2]"
    sc.setLogLevel("ERROR")
    hc = sc._jsc.hadoopConfiguration()
    assert hc.get("fs.azure.account.key.x.blob.core.windows.net") is None
    hc.set("k", "v")
    assert hc.get("k") == "v"


def test_csv_infer_schema(tmp_path, spark):
    p = tmp_path / "d.csv"
    pd.DataFrame({"label": [1, 2, 3], "a": [0.5, 1.5, np.nan], "s": ["x", "y", "z"]}).to_csv(p, index=False)
    sqlc = SQLContext(spark.sparkContext)
    df = sqlc.read.format("com.databricks.spark.csv").options(header="true", inferSchema="true").load(str(p))
    assert df.dtypes == [("label", "int"), ("a", "double"), ("s", "string")]
    assert df.count() == 3
    rows = df.collect()
    assert rows[2].a is None and rows[0]["s"] == "x"
    df2 = spark.read.csv(str(p), header=True)
    assert df2.dtypes[0] == ("label", "string")


def test_select_withcolumn_filter_order(spark):
    pdf = pd.DataFrame({"a": np.arange(10), "b": np.arange(10)[::-1] * 1.5})
    df = spark.createDataFrame(pdf)
    df2 = df.withColumn("c", F.col("a") * 2 + F.col("b")).filter(F.col("a") > 3).orderBy("b", ascending=True)
    ref = pdf.assign(c=pdf.a * 2 + pdf.b)[pdf.a > 3].sort_values("b")
    np.testing.assert_allclose(df2.toPandas()["c"].to_numpy(), ref["c"].to_numpy())
    assert df2.select("a").columns == ["a"]
    assert df.select(F.min("b")).collect()[0][0] == pdf.b.min()
    assert df.select(F.max("a")).collect()[0][0] == 9
    assert df.limit(3).count() == 3
    assert df.orderBy(F.col("a").desc()).first().a == 9


def test_udf_timestamp_and_window_lag_lead(spark):
    # the reference's NYISO feature builder (ddl_nyiso_aztk.py:115-149)
    ts = [(dt.datetime(2016, 1, 2) + dt.timedelta(hours=h)).strftime("%m/%d/%Y %H:%M:%S") for h in range(30)]
    pdf = pd.DataFrame({"TimeStamp": ts[::-1], "Name": ["N.Y.C."] * 30, "v": np.arange(30)[::-1] * 1.0})
    df = spark.createDataFrame(pdf)
    f = F.udf(lambda x: dt.datetime.strptime(x[:19], "%m/%d/%Y %H:%M:%S"), TimestampType())
    df = df.withColumn("TimeStamp", f(F.col("TimeStamp")))
    assert dict(df.dtypes)["TimeStamp"] == "timestamp"
    w = Window.partitionBy("Name").orderBy("TimeStamp")
    for n in (3, 2, 1):
        df = df.withColumn(f"lag{n}", F.lag(F.col("v"), count=n).over(w))
    df = df.withColumn("next1", F.lead(F.col("v"), count=1).over(w))
    out = df.na.drop().orderBy("TimeStamp").toPandas()
    assert len(out) == 30 - 3 - 1
    np.testing.assert_allclose(out["lag3"], out["v"] - 3)
    np.testing.assert_allclose(out["next1"], out["v"] + 1)
    r = df.orderBy("TimeStamp").first()
    assert r.lag1 is None and isinstance(r.TimeStamp, dt.datetime)


def test_window_partitions_are_independent(spark):
    pdf = pd.DataFrame({"g": ["a", "b"] * 5, "t": np.arange(10), "v": np.arange(10) * 1.0})
    df = spark.createDataFrame(pdf)
    w = Window.partitionBy("g").orderBy("t")
    out = df.withColumn("l", F.lag("v", 1).over(w)).withColumn("rn", F.row_number().over(w)).orderBy("t").toPandas()
    assert np.isnan(out.l[0]) and np.isnan(out.l[1])
    np.testing.assert_allclose(out.l[2:], out.v[2:] - 2)
    assert out.rn.tolist() == [1, 1, 2, 2, 3, 3, 4, 4, 5, 5]


def test_repartition_round_robin_and_rdd(spark):
    df = spark.createDataFrame(pd.DataFrame({"a": np.arange(10)}))
    r = df.repartition(3)
    assert r.rdd.getNumPartitions() == 3
    parts = r.rdd.glom().collect()
    assert [len(p[0]) for p in [[p] for p in parts]] == [4, 3, 3]
    assert sorted(x.a for x in r.collect()) == list(range(10))
    assert r.rdd.map(lambda row: row.a).sum() == 45
    assert r.rdd.treeAggregate(0, lambda acc, row: acc + row.a, lambda a, b: a + b, depth=2) == 45
    assert r.coalesce(1).rdd.getNumPartitions() == 1
    counts = r.rdd.mapPartitionsWithIndex(lambda i, it: [(i, sum(1 for _ in it))]).collect()
    assert counts == [(0, 4), (1, 3), (2, 3)]


def test_vector_assembler_and_show(spark, capsys):
    df = spark.createDataFrame(pd.DataFrame({"x": [1.0, 2.0], "y": [3.0, 4.0], "lab": [0, 1]}))
    df = VectorAssembler(inputCols=["x", "y"], outputCol="features").transform(df)
    assert dict(df.dtypes)["features"] == "vector"
    v = df.first().features
    assert isinstance(v, DenseVector) and v.toArray().tolist() == [1.0, 3.0]
    df.show()
    out = capsys.readouterr().out
    assert "|features|" in out.replace(" ", "") and "[1.0,3.0]" in out
    df.printSchema()
    assert "features: vector" in capsys.readouterr().out


def test_rows_and_create_dataframe(spark):
    df = spark.createDataFrame([Row(a=1, b="x"), Row(a=2, b="y")])
    assert df.columns == ["a", "b"] and df.collect()[1].b == "y"
    df2 = spark.createDataFrame([(1, 2.0), (3, 4.0)], ["p", "q"])
    assert df2.groupBy("p").agg(F.sum("q")).count() == 2
    assert spark.range(5).count() == 5
    assert Vectors.sparse(4, [1], [2.0]).toArray().tolist() == [0, 2.0, 0, 0]
    assert SparseVector(3, {0: 1.0}) == DenseVector([1.0, 0, 0])


def test_ml_estimators(spark):
    df = spark.createDataFrame(pd.DataFrame({"c": ["b", "a", "b", "c"], "x": [1.0, 2.0, 3.0, 4.0]}))
    idx = StringIndexer(inputCol="c", outputCol="ci").fit(df).transform(df)
    assert idx.toPandas().ci.tolist() == [0.0, 1.0, 0.0, 2.0]
    oh = OneHotEncoder(inputCol="ci", outputCol="oh").transform(idx)
    assert oh.first().oh.toArray().tolist() == [1.0, 0.0]
    va = VectorAssembler(inputCols=["x"], outputCol="v").transform(df)
    sc = StandardScaler(inputCol="v", outputCol="s", withMean=True).fit(va).transform(va)
    assert abs(sc.toPandas().s.apply(lambda v: v[0]).mean()) < 1e-9


def test_write_read_roundtrip(tmp_path, spark):
    df = spark.createDataFrame(pd.DataFrame({"a": [1, 2, 3], "b": [0.1, 0.2, 0.3]})).repartition(2)
    df.write.mode("overwrite").csv(str(tmp_path / "o"), header=True)
    back = spark.read.csv(str(tmp_path / "o"), header=True, inferSchema=True)
    assert sorted(back.toPandas().a.tolist()) == [1, 2, 3]
    df.write.mode("overwrite").parquet(str(tmp_path / "p"))
    assert spark.read.parquet(str(tmp_path / "p")).count() == 3
    with pytest.raises(IOError):
        spark.read.csv("wasb://container@acct.blob.core.windows.net/x.csv")


from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402


@settings(max_examples=30, deadline=None, derandomize=True, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(n=st.integers(1, 60), groups=st.integers(1, 4), lag=st.integers(1, 5), lead=st.integers(1, 3),
       seed=st.integers(0, 10_000))
def test_window_lag_lead_na_drop_match_pandas(spark, n, groups, lag, lead, seed):
    """Random partitions / orders / offsets: lag & lead over a window, then na.drop, vs pandas."""
    rng = np.random.default_rng(seed)
    pdf = pd.DataFrame({"g": rng.integers(0, groups, n).astype(str), "t": rng.permutation(n),
                        "v": rng.normal(size=n).round(3)})
    df = spark.createDataFrame(pdf)
    w = Window.partitionBy("g").orderBy("t")
    out = df.withColumn("lg", F.lag(F.col("v"), count=lag).over(w)) \
            .withColumn("ld", F.lead(F.col("v"), count=lead).over(w)).na.drop().orderBy("t").toPandas()
    ref = pdf.sort_values("t").copy()
    grp = ref.groupby("g")["v"]
    ref["lg"], ref["ld"] = grp.shift(lag), grp.shift(-lead)
    ref = ref.dropna().sort_values("t")
    assert out["t"].tolist() == ref["t"].tolist()
    np.testing.assert_allclose(out["lg"].to_numpy(), ref["lg"].to_numpy())
    np.testing.assert_allclose(out["ld"].to_numpy(), ref["ld"].to_numpy())
