"""Device ETL kernels (csrc/kernels/ingest.hip) must match the numpy transformers exactly."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture
def spark():
    from distributeddeeplearningspark_amd.context import SparkSession

    return SparkSession.builder.master("local[2]").getOrCreate()


def _col(df, name):
    return np.stack([np.asarray(r[name], dtype=np.float64).reshape(-1) for r in df.collect()])


def test_minmax_onehot_labelindex_on_gpu_match_host(spark):
    from distributeddeeplearningspark_amd.transformers import LabelIndexTransformer, MinMaxTransformer, OneHotTransformer

    rng = np.random.default_rng(0)
    n, K = 1000, 10
    pix = rng.integers(0, 256, (n, 64)).astype(np.float64)
    lab = rng.integers(0, K, n)
    pred = rng.random((n, K))
    pred[5, 3] = pred[5, 7] = 2.0  # tie: first maximum wins
    df = spark.createDataFrame({"pix": list(pix), "label": lab.astype(np.float64), "prediction": list(pred)})
    for dev in (None, "cuda"):
        out = MinMaxTransformer(0.0, 255.0, 0.0, 1.0, "pix", "f", device=dev).transform(df)
        out = OneHotTransformer(K, "label", "oh", device=dev).transform(out)
        out = LabelIndexTransformer(K, device=dev).transform(out)
        res = (_col(out, "f"), _col(out, "oh"), _col(out, "prediction_index"))
        if dev is None:
            host = res
    for a, b in zip(host, res):
        np.testing.assert_array_equal(a, b)
    assert res[2][5, 0] == 3.0


def test_onehot_out_of_range_raises_on_gpu(spark):
    from distributeddeeplearningspark_amd.transformers import OneHotTransformer

    df = spark.createDataFrame({"label": [1.0, 12.0]})
    with pytest.raises(ValueError):
        OneHotTransformer(10, "label", "oh", device="cuda").transform(df)
