"""hipGraph-captured training steps (models/step.py) must train exactly like the eager step,
and co-located dist-keras workers (DDL_WORKERS_PER_GPU) must follow the update law."""
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _train(build, opt, loss, x, y, steps, graphs, monkeypatch):
    from distributeddeeplearningspark_amd.models.step import CompiledTrainStep

    monkeypatch.setenv("DDL_GRAPHS", "1" if graphs else "0")
    m = build()
    m.compile(opt, loss)
    m.place("cuda:0", seed=3)
    st = CompiledTrainStep(m)
    xs, ys = m.to_input(x), m.to_target(y)
    bs = x.shape[0] // steps
    out = []
    for i in range(steps):
        out.append(float(st(xs[i * bs:(i + 1) * bs], ys[i * bs:(i + 1) * bs])))
    torch.cuda.synchronize()
    assert st.captured == graphs, st.fallback_reason
    return np.array(out), m.arena.master.detach().cpu().clone(), m.optimizer.iterations


@pytest.mark.parametrize("which", ["gru-adagrad", "lstm-adam", "mnist-adam"])
def test_graph_step_matches_eager(which, monkeypatch):
    from distributeddeeplearningspark_amd.models import zoo

    g = torch.Generator().manual_seed(0)
    steps = 8
    if which == "mnist-adam":
        build, opt, loss = zoo.mnist_cnn, "adam", "categorical_crossentropy"
        x = torch.rand(16 * steps, 28, 28, 1, generator=g).numpy()
        y = torch.nn.functional.one_hot(torch.randint(0, 10, (16 * steps,), generator=g), 10).float().numpy()
    else:
        build = zoo.gru_regressor if which.startswith("gru") else zoo.lstm_regressor
        opt = which.split("-")[1]
        loss = "mean_squared_error"
        x = torch.rand(32 * steps, 25, 1, generator=g).numpy()
        y = torch.rand(32 * steps, 1, generator=g).numpy()
    le, we, ie = _train(build, opt, loss, x, y, steps, False, monkeypatch)
    lg, wg, ig = _train(build, opt, loss, x, y, steps, True, monkeypatch)
    assert ie == ig == steps
    assert np.allclose(le, lg, rtol=2e-3, atol=1e-5), (le, lg)
    rel = ((we - wg).norm() / we.norm()).item()
    assert rel < 2e-3, rel


def test_graph_step_is_faster_than_eager(monkeypatch):
    """The point of the graph: a GRU(128) step at batch 32 is launch-bound when eager."""
    from distributeddeeplearningspark_amd.models import zoo
    from distributeddeeplearningspark_amd.models.step import CompiledTrainStep

    res = {}
    for graphs in (False, True):
        monkeypatch.setenv("DDL_GRAPHS", "1" if graphs else "0")
        m = zoo.gru_regressor()
        m.compile("adagrad", "mean_squared_error")
        m.place("cuda:0", seed=0)
        st = CompiledTrainStep(m)
        x = m.to_input(torch.rand(32, 25, 1))
        y = m.to_target(torch.rand(32, 1))
        for _ in range(5):
            st(x, y)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(200):
            st(x, y)
        torch.cuda.synchronize()
        res[graphs] = (time.perf_counter() - t0) / 200
    print(f"GRU step: eager {res[False] * 1e6:.0f} us, hipGraph {res[True] * 1e6:.0f} us")
    assert res[True] < res[False] * 1.15  # GPU-bound once the recurrences are fast; never slower


def test_colocated_workers_follow_update_law(monkeypatch):
    """Two ADAG workers sharing one MI355X (gloo, host-staged commits)."""
    from distributeddeeplearningspark_amd.context import SparkSession
    from distributeddeeplearningspark_amd.models import zoo
    from distributeddeeplearningspark_amd.trainers import ADAG

    monkeypatch.setenv("DDL_WORKERS_PER_GPU", "2")
    rng = np.random.default_rng(0)
    n = 640
    X = rng.random((n, 25, 1)).astype(np.float32)
    Y = X[:, -4:, 0].mean(1, keepdims=True).astype(np.float32)
    spark = SparkSession.builder.master("local[2]").getOrCreate()
    df = spark.createDataFrame({"x": list(X), "y": list(Y)})
    tr = ADAG(keras_model=zoo.gru_regressor(), worker_optimizer="adagrad", loss="mean_squared_error", num_workers=2,
              batch_size=32, communication_window=5, num_epoch=2, features_col="x", label_col="y", device="cuda")
    tr.train(df.repartition(2))
    # 320 rows per worker -> 10 batches/epoch -> 20 steps -> 4 commits per worker
    assert tr.parameter_server.num_updates == 8
    h = tr.get_history()
    assert len(h) > 0 and np.isfinite(np.asarray(h, dtype=np.float64)).all()
