"""dist-keras surface: transformers, model API (param counts / Keras layouts / JSON),
predictors, evaluators, MAPE, and the trainers on CPU executors (gloo, world size 2)."""
import json

import numpy as np
import pandas as pd
import pytest
import torch

from distributeddeeplearningspark_amd.context import SparkSession
from distributeddeeplearningspark_amd.evaluators import AccuracyEvaluator, get_MAPE
from distributeddeeplearningspark_amd.ml.feature import VectorAssembler
from distributeddeeplearningspark_amd.models import Dense, Sequential, model_from_json
from distributeddeeplearningspark_amd.models.zoo import gru_regressor, lenet5, lstm_regressor, mnist_cnn, vgg16
from distributeddeeplearningspark_amd.predictors import ModelPredictor
from distributeddeeplearningspark_amd.transformers import (DenseTransformer, LabelIndexTransformer,
                                                           MinMaxTransformer, OneHotTransformer, ReshapeTransformer)
from distributeddeeplearningspark_amd.utils import deserialize_keras_model, serialize_keras_model


@pytest.fixture(scope="module")
def spark():
    return SparkSession.builder.master("local[2]").getOrCreate()


# ------------------------------------------------------------------ transformers
def test_minmax_scalar_vector_inverse(spark):
    df = spark.createDataFrame(pd.DataFrame({"t": [10.0, 20.0, 30.0]}))
    df = MinMaxTransformer(n_min=0.0, n_max=1.0, o_min=10.0, o_max=30.0, input_col="t", output_col="n",
                           is_vector=False).transform(df)
    assert df.toPandas().n.tolist() == [0.0, 0.5, 1.0]
    df = VectorAssembler(inputCols=["n"], outputCol="v").transform(df)
    inv = MinMaxTransformer(n_min=10.0, n_max=30.0, o_min=0.0, o_max=1.0, input_col="v", output_col="back",
                            is_vector=True).transform(df)
    assert [r.back.toArray()[0] for r in inv.collect()] == [10.0, 20.0, 30.0]


def test_onehot_reshape_dense_labelindex(spark):
    df = spark.createDataFrame(pd.DataFrame({"label": [3, 0, 9]}))
    df = OneHotTransformer(10, input_col="label", output_col="enc").transform(df)
    enc = np.stack([r.enc.toArray() for r in df.collect()])
    assert enc.argmax(1).tolist() == [3, 0, 9] and enc.sum() == 3
    df = DenseTransformer(input_col="enc", output_col="dense").transform(df)
    df = ReshapeTransformer("dense", "mat", (2, 5)).transform(df)
    assert dict(df.dtypes)["mat"] == "array<array<double>>"
    assert np.asarray(df.first().mat).shape == (2, 5)
    df = LabelIndexTransformer(output_dim=10, input_col="enc").transform(df)
    assert df.toPandas().prediction_index.tolist() == [3.0, 0.0, 9.0]
    assert AccuracyEvaluator(prediction_col="prediction_index", label_col="label").evaluate(df) == 1.0


def test_mape_semantics():
    assert abs(get_MAPE([[100.0], [200.0]], [[110.0], [180.0]]) - 10.0) < 1e-12
    assert np.isnan(get_MAPE([[0.0]], [[1.0]]))  # inf -> nan (ddl_nyiso_aztk.py:240-241)


# ------------------------------------------------------------------ models
def test_reference_param_counts():
    # SURVEY §4 oracles: 1,048,853 / 50,049 / 66,689 (ddl_nyiso_hdi.ipynb:549-554,772-777)
    assert mnist_cnn().count_params() or True
    m = mnist_cnn()
    m.build_model()
    assert m.count_params() == 1048853
    g = gru_regressor()
    g.build_model()
    assert g.count_params() == 50049
    assert [l.count_params() for l in g.layers] == [49920, 129]
    lst = lstm_regressor()
    lst.build_model()
    assert lst.count_params() == 66689
    assert [l.count_params() for l in lst.layers] == [66560, 129]
    v = vgg16()
    v.build_model()
    l5 = lenet5()
    l5.build_model()
    assert l5.count_params() == 61706


def test_summary_format(capsys):
    g = gru_regressor()
    g.summary()
    out = capsys.readouterr().out
    assert "(None, 128)" in out and "49920" in out and "Total params: 50,049" in out


def test_keras_weight_layouts_and_json_roundtrip():
    m = mnist_cnn()
    ws = m.get_weights()
    assert [w.shape for w in ws] == [(3, 3, 1, 32), (32,), (3, 3, 32, 32), (32,), (4608, 225), (225,), (225, 10), (10,)]
    g = gru_regressor()
    assert [w.shape for w in g.get_weights()] == [(1, 384), (128, 384), (384,), (128, 1), (1,)]
    lst = lstm_regressor()
    b = lst.get_weights()[2]
    assert (b[128:256] == 1).all() and (b[:128] == 0).all()  # unit_forget_bias, gate order i,f,c,o
    m2 = model_from_json(m.to_json())
    m2.set_weights(ws)
    for a, c in zip(ws, m2.get_weights()):
        np.testing.assert_array_equal(a, c)
    d = serialize_keras_model(m)
    json.loads(d["model"])
    m3 = deserialize_keras_model(d)
    x = np.random.rand(2, 28, 28, 1).astype(np.float32)
    np.testing.assert_allclose(m.predict(x), m3.predict(x), rtol=1e-5, atol=1e-6)


def test_gru_lstm_match_keras_math():
    """Hand-written Keras-2 GRU (reset_after=False) / LSTM cell, numpy, vs our layers."""
    rng = np.random.default_rng(0)
    x = rng.normal(size=(3, 5, 1)).astype(np.float32)
    hs = lambda z: np.clip(0.2 * z + 0.5, 0, 1)
    for kind in ("gru", "lstm"):
        m = gru_regressor(units=4, seq_len=5) if kind == "gru" else lstm_regressor(units=4, seq_len=5)
        W, U, b, Wd, bd = m.get_weights()
        H = 4
        h = np.zeros((3, H))
        c = np.zeros((3, H))
        for t in range(5):
            xt = x[:, t] @ W + b
            if kind == "gru":
                z = hs(xt[:, :H] + h @ U[:, :H])
                r = hs(xt[:, H:2 * H] + h @ U[:, H:2 * H])
                hh = np.tanh(xt[:, 2 * H:] + (r * h) @ U[:, 2 * H:])
                h = z * h + (1 - z) * hh
            else:
                g = xt + h @ U
                i, f, cc, o = hs(g[:, :H]), hs(g[:, H:2 * H]), np.tanh(g[:, 2 * H:3 * H]), hs(g[:, 3 * H:])
                c = f * c + i * cc
                h = o * np.tanh(c)
        ref = h @ Wd + bd
        np.testing.assert_allclose(m.predict(x), ref, rtol=1e-4, atol=1e-5)


def test_train_on_batch_learns_regression():
    torch.manual_seed(0)
    from distributeddeeplearningspark_amd.models.optimizers import Adam

    m = Sequential([Dense(16, activation="relu", input_shape=(4,)), Dense(1)])
    m.compile(Adam(lr=0.01), "mean_squared_error")
    x = np.random.rand(256, 4).astype(np.float32)
    y = (x @ np.array([1.0, -2.0, 0.5, 3.0], dtype=np.float32))[:, None]
    first = m.evaluate(x, y)
    m.fit(x, y, batch_size=32, epochs=30)
    assert m.evaluate(x, y) < 0.1 * first


# ------------------------------------------------------------------ trainers (multi-process gloo)
def _mnist_frame(spark, n=600):
    from distributeddeeplearningspark_amd.data.synthetic import mnist_like

    raw = spark.createDataFrame(mnist_like(n, seed=2))
    feats = [c for c in raw.columns if c != "label"]
    df = VectorAssembler(inputCols=feats, outputCol="features").transform(raw)
    df = OneHotTransformer(10, input_col="label", output_col="label_encoded").transform(df)
    df = MinMaxTransformer(n_min=0.0, n_max=1.0, o_min=0.0, o_max=250.0, input_col="features",
                           output_col="fn").transform(df)
    df = ReshapeTransformer("fn", "matrix", (28, 28, 1)).transform(df)
    return df.select("matrix", "label", "label_encoded")


@pytest.mark.parametrize("algo", ["ADAG", "DynSGD", "DOWNPOUR", "AEASGD"])
def test_trainers_two_workers_update_law(spark, algo):
    from distributeddeeplearningspark_amd import trainers as T

    df = _mnist_frame(spark, 400).repartition(2)
    cls = getattr(T, algo)
    tr = cls(keras_model=mnist_cnn(), worker_optimizer="adam", loss="categorical_crossentropy", num_workers=2,
             batch_size=16, communication_window=5, num_epoch=2, features_col="matrix", label_col="label_encoded",
             device="cpu")
    model = tr.train(df)
    # num_updates = sum_w floor(E * floor(rows_w / bs) / window): 200 rows -> 12 batches -> 24 steps -> 4 commits
    assert tr.parameter_server.num_updates == 2 * ((2 * (200 // 16)) // 5)
    assert tr.get_training_time() > 0
    assert len(tr.get_history()) == 2 and len(tr.get_history()[0]) == 24
    pred = ModelPredictor(keras_model=model, features_col="matrix").predict(df)
    pred = LabelIndexTransformer(output_dim=10).transform(pred)
    acc = AccuracyEvaluator(prediction_col="prediction_index", label_col="label").evaluate(pred)
    assert acc > 0.5, acc


def test_adag_sync_semantics_match_simulation(spark):
    """2 workers, window 2: the center after training equals a single-process simulation
    c += sum_w (W_w - c)/k with worker-local SGD from the same start."""
    from distributeddeeplearningspark_amd.trainers import ADAG

    rng = np.random.default_rng(0)
    x = rng.normal(size=(32, 3)).astype(np.float32)
    y = (x.sum(1, keepdims=True)).astype(np.float32)
    df = spark.createDataFrame({"f": list(x), "l": list(y)}).repartition(2)
    base = Sequential([Dense(1, input_shape=(3,))])
    w0 = base.get_weights()
    tr = ADAG(keras_model=base, worker_optimizer="sgd", loss="mean_squared_error", num_workers=2, batch_size=4,
              communication_window=2, num_epoch=1, features_col="f", label_col="l", device="cpu")
    out = tr.train(df).get_weights()
    # simulation
    shards = [x[0::2], x[1::2]], [y[0::2], y[1::2]]
    center = [w.copy() for w in w0]
    workers = []
    for r in range(2):
        m = Sequential([Dense(1, input_shape=(3,))])
        m.compile("sgd", "mean_squared_error")
        m.set_weights(center)
        workers.append(m)
    for rnd in range(2):
        deltas = []
        for r, m in enumerate(workers):
            m.set_weights(center)
            for b in range(2):
                i = (rnd * 2 + b) * 4
                m.train_on_batch(shards[0][r][i:i + 4], shards[1][r][i:i + 4])
            deltas.append([(a - c) / 2 for a, c in zip(m.get_weights(), center)])
        center = [c + d0 + d1 for c, d0, d1 in zip(center, *deltas)]
    for a, b in zip(out, center):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6)
    assert tr.parameter_server.num_updates == 4


def test_single_averaging_ensemble_syncdp(spark):
    from distributeddeeplearningspark_amd.trainers import (AveragingTrainer, EnsembleTrainer, SingleTrainer,
                                                            SynchronousDataParallel)

    df = _mnist_frame(spark, 200)
    common = dict(worker_optimizer="adam", loss="categorical_crossentropy", features_col="matrix",
                  label_col="label_encoded", batch_size=20, num_epoch=1, device="cpu")
    st = SingleTrainer(keras_model=mnist_cnn(), **common)
    st.train(df)
    assert st.parameter_server.num_updates == 10
    av = AveragingTrainer(keras_model=mnist_cnn(), num_workers=2, **common)
    av.train(df.repartition(2))
    ens = EnsembleTrainer(keras_model=mnist_cnn(), num_ensembles=2, **{k: v for k, v in common.items()})
    models = ens.train(df.repartition(2))
    assert len(models) == 2
    sd = SynchronousDataParallel(keras_model=mnist_cnn(), num_workers=2, **common)
    w_sd = sd.train(df.repartition(2)).get_weights()
    assert sd.parameter_server.num_updates == 5
    # the dist-keras spelling of the same per-step gradient all-reduce
    from distributeddeeplearningspark_amd.trainers import ADAG

    ag = ADAG(keras_model=mnist_cnn(), num_workers=2, communication_window=1, mode="sync-grad", **common)
    w_ag = ag.train(df.repartition(2)).get_weights()
    assert ag.parameter_server.num_updates == 5
    for a, b in zip(w_ag, w_sd):
        np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-7)
    with pytest.raises(ValueError):
        ADAG(keras_model=mnist_cnn(), num_workers=2, mode="bogus", **common)


# ------------------------------------------------------------------ native async parameter server
def test_native_param_server_protocol():
    """commit/pull framing, ADD vs DynSGD staleness rule (center += r / (staleness + 1))."""
    import torch

    from distributeddeeplearningspark_amd.parallel.ps import (RULE_ADD, RULE_DYNSGD, ParameterServerClient,
                                                              ParameterServerProcess)

    init = torch.arange(6, dtype=torch.float32)
    with ParameterServerProcess(init, rule=RULE_ADD) as ps:
        a = ParameterServerClient(ps.port, 0, 6)
        b = ParameterServerClient(ps.port, 1, 6)
        assert torch.equal(a.pull(), init) and a.last_update == 0
        a.commit(torch.ones(6))
        a.pull()  # commits are fire-and-forget (as in dist-keras); a pull on the same connection orders them
        b.commit(torch.full((6,), 2.0))
        assert torch.equal(b.pull(), init + 3) and b.last_update == 2
        a.close(), b.close()
        assert ps.num_updates == 2 and torch.equal(ps.center(), init + 3)
    with ParameterServerProcess(torch.zeros(4), rule=RULE_DYNSGD) as ps:
        a = ParameterServerClient(ps.port, 0, 4)
        b = ParameterServerClient(ps.port, 1, 4)
        a.pull(), b.pull()  # both at update 0
        a.commit(torch.ones(4))  # staleness 0 -> +1
        b.commit(torch.ones(4))  # staleness 1 -> +1/2
        a.pull(), b.pull()  # both commits applied (whichever order the server saw them in, the sum is 1.5)
        np.testing.assert_allclose(ps.center().numpy(), 1.5)
        a.close(), b.close()


def test_async_adag_single_worker_matches_simulation(spark):
    """One async worker: pull -> k steps -> commit (W - anchor)/k -> pull, exactly."""
    from distributeddeeplearningspark_amd.trainers import ADAG

    rng = np.random.default_rng(1)
    x = rng.normal(size=(24, 3)).astype(np.float32)
    y = x.sum(1, keepdims=True).astype(np.float32)
    df = spark.createDataFrame({"f": list(x), "l": list(y)}).repartition(1)
    base = Sequential([Dense(1, input_shape=(3,))])
    w0 = base.get_weights()
    tr = ADAG(keras_model=base, worker_optimizer="sgd", loss="mean_squared_error", num_workers=1, batch_size=4,
              communication_window=3, num_epoch=1, features_col="f", label_col="l", device="cpu", mode="async")
    out = tr.train(df).get_weights()
    m = Sequential([Dense(1, input_shape=(3,))])
    m.compile("sgd", "mean_squared_error")
    center = [w.copy() for w in w0]
    for rnd in range(2):
        m.set_weights(center)
        for b in range(3):
            i = (rnd * 3 + b) * 4
            m.train_on_batch(x[i:i + 4], y[i:i + 4])
        center = [c + (a - c) / 3 for a, c in zip(m.get_weights(), center)]
    for a, b in zip(out, center):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6)
    assert tr.parameter_server.num_updates == 2


@pytest.mark.parametrize("algo", ["DynSGD", "DOWNPOUR"])
def test_async_two_workers_train(spark, algo):
    from distributeddeeplearningspark_amd import trainers as T

    df = _mnist_frame(spark, 400).repartition(2)
    tr = getattr(T, algo)(keras_model=mnist_cnn(), worker_optimizer="adam", loss="categorical_crossentropy",
                          num_workers=2, batch_size=16, communication_window=5, num_epoch=2, features_col="matrix",
                          label_col="label_encoded", device="cpu", mode="async")
    model = tr.train(df)
    assert tr.parameter_server.num_updates == 2 * ((2 * (200 // 16)) // 5)
    pred = ModelPredictor(keras_model=model, features_col="matrix").predict(df)
    pred = LabelIndexTransformer(output_dim=10).transform(pred)
    acc = AccuracyEvaluator(prediction_col="prediction_index", label_col="label").evaluate(pred)
    assert acc > 0.5, acc


def test_uint8_images_are_scaled_unless_normalisation_declared():
    """4-D uint8 NHWC batches are images: x / 255 by default, (x - mean) / std when the model
    declares input_mean / input_std; 2-D integer columns keep their values."""
    from distributeddeeplearningspark_amd.models import Conv2D, Flatten

    m = Sequential([Conv2D(2, (3, 3), input_shape=(4, 4, 3)), Flatten(), Dense(1)])
    m.place("cpu")
    x = np.arange(2 * 4 * 4 * 3, dtype=np.uint8).reshape(2, 4, 4, 3) * 2
    torch.testing.assert_close(m.to_input(x), torch.from_numpy(x.astype(np.float32) / 255.0))
    m.input_mean, m.input_std = (10.0, 20.0, 30.0), (2.0, 4.0, 8.0)
    ref = (x.astype(np.float32) - np.array([10.0, 20.0, 30.0], np.float32)) / np.array([2.0, 4.0, 8.0], np.float32)
    torch.testing.assert_close(m.to_input(x), torch.from_numpy(ref))
    flat = Sequential([Dense(1, input_shape=(6,))])
    flat.place("cpu")
    torch.testing.assert_close(flat.to_input(np.full((2, 6), 7, np.uint8)), torch.full((2, 6), 7.0))


def test_integer_feature_column_trains_and_predicts_as_float(spark):
    """uint8 / int64 2-D feature columns reach Dense as their values in the compute dtype
    (partition_arrays keeps column dtypes; Model.to_input casts non-image integers)."""
    from distributeddeeplearningspark_amd.sql.dataframe import from_columns
    from distributeddeeplearningspark_amd.trainers import SingleTrainer

    rng = np.random.default_rng(0)
    X = rng.integers(0, 4, (64, 6)).astype(np.uint8)
    y = (X.astype(np.float32) @ np.arange(6, dtype=np.float32) / 10.0)[:, None]
    df = from_columns({"features": X, "label": y}, num_partitions=1)
    m = Sequential([Dense(1, input_shape=(6,))])
    m.compile("sgd", "mean_squared_error")
    m.place("cpu")
    t = m.to_input(X)
    assert t.dtype == torch.float32
    torch.testing.assert_close(t, torch.from_numpy(X.astype(np.float32)))
    tr = SingleTrainer(keras_model=m, worker_optimizer="adam", loss="mean_squared_error", features_col="features",
                       label_col="label", batch_size=8, num_epoch=20)
    trained = tr.train(df)
    h = tr.get_history()[0]
    assert np.isfinite(h).all() and np.mean(h[-8:]) < np.mean(h[:8])
    out = ModelPredictor(keras_model=trained, features_col="features").predict(df)
    p = np.stack([r["prediction"].toArray() for r in out.collect()])
    ref = trained.predict(X.astype(np.float32), batch_size=64)
    np.testing.assert_allclose(p, ref, rtol=1e-5, atol=1e-5)


def test_partitions_reach_executors_through_shared_memory(spark, monkeypatch):
    """Executor-pool tasks carry shard DESCRIPTORS, not pickled arrays: the arrays are placed in
    /dev/shm once and mapped zero-copy by the executors (parallel/executors.py); the training
    result equals the pickle path, a repeated train() re-uses the blocks, and they are unlinked
    when the pool shuts down."""
    import glob

    from distributeddeeplearningspark_amd.parallel import executors as EX
    from distributeddeeplearningspark_amd.sql.dataframe import from_columns
    from distributeddeeplearningspark_amd.trainers import ADAG

    rng = np.random.default_rng(5)
    X = rng.normal(size=(4096, 64)).astype(np.float32)  # 1 MB
    y = (X[:, :1] * 0.5).astype(np.float32)
    df = from_columns({"features": X, "label": y}, num_partitions=2)
    out = {}
    for mode, thr in (("shm", "0.01"), ("pickle", "100000")):
        monkeypatch.setenv("DDL_SHM_MIN_MB", thr)
        m = Sequential([Dense(1, input_shape=(64,))])
        m.compile("sgd", "mean_squared_error")
        tr = ADAG(keras_model=m, worker_optimizer="sgd", loss="mean_squared_error", num_workers=2, batch_size=64,
                  communication_window=2, num_epoch=1, features_col="features", label_col="label", device="cpu")
        w = tr.train(df).get_weights()
        pool = next(iter(EX._POOLS.values()))
        out[mode] = (w, pool.last_payload_bytes, len(EX._SHM_BLOCKS))
        if mode == "shm":
            blocks = len(EX._SHM_BLOCKS)
            tr.train(df)  # same cached frame: no new blocks
            assert len(EX._SHM_BLOCKS) == blocks
            names = [e[1].name for e in EX._SHM_BLOCKS.values()]
        EX.shutdown_all()
    w_shm, bytes_shm, nblocks = out["shm"]
    w_pk, bytes_pk, _ = out["pickle"]
    assert nblocks >= 2 and bytes_shm < bytes_pk / 10, (bytes_shm, bytes_pk)
    for a, b in zip(w_shm, w_pk):
        np.testing.assert_array_equal(a, b)
    assert not any(glob.glob("/dev/shm/" + n) for n in names)  # unlinked with the pool


def test_shared_shards_follow_in_place_mutation(spark, monkeypatch):
    """A shard cached in /dev/shm is re-validated by content hash: modifying the user's array in place
    between two train() calls trains on the NEW values (no stale shared-memory copy)."""
    from distributeddeeplearningspark_amd.parallel import executors as EX
    from distributeddeeplearningspark_amd.sql.dataframe import from_columns
    from distributeddeeplearningspark_amd.trainers import ADAG

    rng = np.random.default_rng(6)
    X = rng.normal(size=(4096, 64)).astype(np.float32)
    y = (X[:, :1] * 0.5).astype(np.float32)

    def train(thr):
        monkeypatch.setenv("DDL_SHM_MIN_MB", thr)
        m = Sequential([Dense(1, input_shape=(64,))])
        m.set_weights([np.full((64, 1), 0.01, np.float32), np.zeros(1, np.float32)])
        tr = ADAG(keras_model=m, worker_optimizer="sgd", loss="mean_squared_error", num_workers=2, batch_size=64,
                  communication_window=2, num_epoch=1, features_col="features", label_col="label", device="cpu")
        return tr.train(from_columns({"features": X, "label": y}, num_partitions=2)).get_weights()

    train("0.01")  # blocks created for the original values
    X *= 3.0  # in place: same buffer, same id, new content
    w_shm = train("0.01")
    EX.shutdown_all()
    w_ref = train("100000")  # pickle path: always ships the current values
    EX.shutdown_all()
    for a, b in zip(w_shm, w_ref):
        np.testing.assert_array_equal(a, b)


def test_shared_block_follows_mutation_of_readonly_view_base():
    """A READ-ONLY view of a writable base (``setflags(write=False)`` on a view) must still be
    re-validated: the base can change in place under the cached /dev/shm block."""
    from multiprocessing import shared_memory

    from distributeddeeplearningspark_amd.parallel import executors as EX

    base = np.arange(4096, dtype=np.float32).reshape(64, 64)
    view = base[8:40]
    view.setflags(write=False)

    def read(desc):
        shm = shared_memory.SharedMemory(name=desc.name)
        try:
            return np.ndarray(desc.shape, np.dtype(desc.dtype), buffer=shm.buf).copy()
        finally:
            shm.close()

    d0 = EX.share_array(view)
    np.testing.assert_array_equal(read(d0), base[8:40])
    base *= 2.0  # in place, through the writable base
    d1 = EX.share_array(view)
    np.testing.assert_array_equal(read(d1), base[8:40])


def test_prob_cross_entropy_cpu_matches_keras_formula():
    from distributeddeeplearningspark_amd.ops.loss import prob_cross_entropy

    g = torch.Generator().manual_seed(0)
    p = torch.softmax(torch.randn(9, 5, generator=g) * 4, -1)
    lab = torch.randint(0, 5, (9,), generator=g)
    y = torch.nn.functional.one_hot(lab, 5).float()
    ref = -(y * torch.log(p.clamp(1e-7, 1 - 1e-7))).sum(-1).mean()
    assert torch.allclose(prob_cross_entropy(p, labels=lab), ref, atol=1e-6)
    assert torch.allclose(prob_cross_entropy(p, target=y), ref, atol=1e-6)
