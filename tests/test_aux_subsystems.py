"""Auxiliary subsystems: checkpoint/resume, tracing, metrics, watchdog,
fault injection + restart, replica divergence check."""
import json
import os
import time

import numpy as np
import pytest
import torch

from distributeddeeplearningspark_amd.models import Dense, Sequential
from distributeddeeplearningspark_amd.models.zoo import mnist_cnn


def _reg_model():
    m = Sequential([Dense(16, activation="relu", input_shape=(4,)), Dense(1)])
    m.compile("adam", "mean_squared_error")
    m.place("cpu", seed=0)
    return m


def test_checkpoint_roundtrip_and_exact_resume(tmp_path):
    from distributeddeeplearningspark_amd.utils.checkpoint import (latest_checkpoint, load_checkpoint,
                                                                   load_keras_weights, save_checkpoint)

    rng = np.random.default_rng(0)
    x = rng.normal(size=(64, 4)).astype(np.float32)
    y = x.sum(1, keepdims=True)
    a = _reg_model()
    for _ in range(3):
        a.train_on_batch(x, y)
    for s in (3, 4, 5, 6):
        save_checkpoint(str(tmp_path), a, step=s, keep=2)
    assert sorted(os.listdir(tmp_path)) == ["latest", "step_000000005", "step_000000006"]
    path = latest_checkpoint(str(tmp_path))
    ws = load_keras_weights(path)
    for w0, w1 in zip(a.get_weights(), ws):
        np.testing.assert_array_equal(w0, w1)
    b, meta = load_checkpoint(str(tmp_path), device="cpu")  # rebuilt from model.json
    assert meta["step"] == 6 and b.optimizer.iterations == a.optimizer.iterations
    la = [a.train_on_batch(x, y) for _ in range(3)]
    lb = [b.train_on_batch(x, y) for _ in range(3)]
    np.testing.assert_allclose(la, lb, rtol=1e-6)


def test_tracer_chrome_json_and_step_timer(tmp_path):
    from distributeddeeplearningspark_amd.utils.tracing import StepTimer, Tracer, trace_range

    with Tracer() as t:
        with trace_range("step"):
            with trace_range("fwd"):
                time.sleep(0.002)
    p = t.dump(str(tmp_path / "trace.json"))
    ev = json.load(open(p))["traceEvents"]
    names = {e["name"] for e in ev}
    assert {"step", "fwd"} <= names
    fwd = next(e for e in ev if e["name"] == "fwd")
    assert fwd["dur"] >= 1000  # us
    st = StepTimer("cpu")
    with st.phase("a"):
        time.sleep(0.001)
    assert st.summary()["a"] >= 1.0


def test_metrics_jsonl(tmp_path):
    from distributeddeeplearningspark_amd.utils.metrics import MetricsLogger, read_jsonl

    ml = MetricsLogger(str(tmp_path / "m.jsonl"), rank=0)
    for s in range(3):
        ml.log(s, samples=32, loss=1.0 / (s + 1), phases={"allreduce": 2.0}, comm_bytes=4_000_000)
    ml.close()
    recs = read_jsonl(str(tmp_path / "m.jsonl"))
    assert len(recs) == 3 and recs[1]["loss"] == 0.5 and recs[0]["allreduce_GBps"] == 2.0


def test_watchdog_fires_on_stall():
    from distributeddeeplearningspark_amd.utils.fault import Watchdog

    hit = []
    w = Watchdog(timeout_s=0.3, on_timeout=lambda: hit.append(1)).start()
    for _ in range(3):
        time.sleep(0.1)
        w.beat()
    assert not w.fired
    time.sleep(1.0)
    w.stop()
    assert w.fired and hit == [1]


def _mnist_df(spark, n=256):
    from distributeddeeplearningspark_amd.data.synthetic import mnist_like
    from distributeddeeplearningspark_amd.ml.feature import VectorAssembler
    from distributeddeeplearningspark_amd.transformers import OneHotTransformer, ReshapeTransformer

    raw = spark.createDataFrame(mnist_like(n, seed=3))
    feats = [c for c in raw.columns if c != "label"]
    df = VectorAssembler(inputCols=feats, outputCol="f").transform(raw)
    df = OneHotTransformer(10, input_col="label", output_col="y").transform(df)
    return ReshapeTransformer("f", "x", (28, 28, 1)).transform(df).select("x", "y")


@pytest.fixture
def spark():
    from distributeddeeplearningspark_amd.context import SparkSession

    s = SparkSession.builder.master("local[2]").getOrCreate()
    yield s
    s.stop()


def test_fault_injection_restart_resumes_from_checkpoint(spark, tmp_path, monkeypatch, capfd):
    """Rank 1 dies at step 7 of the first attempt; the launcher restarts both workers,
    which resume from the last commit-round checkpoint and finish with the full update law."""
    from distributeddeeplearningspark_amd.trainers import ADAG

    monkeypatch.setenv("DDL_FAULT_RANK", "1")
    monkeypatch.setenv("DDL_FAULT_STEP", "7")
    df = _mnist_df(spark).repartition(2)
    tr = ADAG(keras_model=mnist_cnn(), worker_optimizer="adam", loss="categorical_crossentropy", num_workers=2,
              batch_size=16, communication_window=2, num_epoch=1, features_col="x", label_col="y", device="cpu",
              checkpoint_dir=str(tmp_path), checkpoint_every=1, max_restarts=1)
    tr.train(df)
    out = capfd.readouterr()
    assert "injecting 'exit' on rank 1 at step 7" in out.err
    assert "restarting all workers" in out.out
    assert tr.parameter_server.num_updates == 2 * ((128 // 16) // 2)
    assert any(d.startswith("step_") for d in os.listdir(tmp_path))
    # resumed attempt skipped the 6 batches done before the last checkpoint
    assert len(tr.get_history()[0]) == 8 - 6


def _replica_worker(rank, world, pg):
    from distributeddeeplearningspark_amd.parallel.ddp import DataParallel

    m = _reg_model()
    ddp = DataParallel(m, pg)
    ddp.broadcast_parameters()
    x = torch.randn(8, 4) + rank
    ddp.train_step(x, x.sum(1, keepdim=True))
    ok1 = ddp.check_replicas()
    if rank == 1:
        with torch.no_grad():
            m.arena.master[0] += 1.0
    ok2 = ddp.check_replicas(raise_on_mismatch=False)
    return ok1, ok2


def test_ddp_replica_checksums_gloo():
    from distributeddeeplearningspark_amd.parallel.launcher import run_workers

    res = run_workers(_replica_worker, 2, [()] * 2, device="cpu")
    assert res == [(True, False), (True, False)]


def _pid_env_worker(rank, world, pg):
    import os

    return os.getpid(), os.environ.get("DDL_TEST_KNOB")


def _fail_once_worker(rank, world, pg):
    import os

    if rank == 1 and os.environ.get("DDL_RESTART_COUNT") == "0":
        raise RuntimeError("boom")
    return os.getpid()


def test_executor_pool_is_reused_and_forwards_env(monkeypatch):
    """Executors are long-lived (Spark executor analog): the second job runs in the same
    processes, sees DDL_* variables set after the pool started, and a failed task tears the
    pool down so the restart runs on fresh executors."""
    from distributeddeeplearningspark_amd.parallel.executors import shutdown_all
    from distributeddeeplearningspark_amd.parallel.launcher import run_workers

    shutdown_all()
    a = run_workers(_pid_env_worker, 2, [()] * 2, device="cpu")
    monkeypatch.setenv("DDL_TEST_KNOB", "42")
    b = run_workers(_pid_env_worker, 2, [()] * 2, device="cpu")
    assert [p for p, _ in a] == [p for p, _ in b]
    assert [k for _, k in a] == [None, None] and [k for _, k in b] == ["42", "42"]
    pids = run_workers(_fail_once_worker, 2, [()] * 2, device="cpu", max_restarts=1)
    assert set(pids).isdisjoint(p for p, _ in a)


def test_spark_context_prestarts_executors():
    from distributeddeeplearningspark_amd.context import SparkConf, SparkContext
    from distributeddeeplearningspark_amd.parallel import executors as E

    E.shutdown_all()
    conf = SparkConf().set("spark.master", "local[2]").set("spark.executor.instances", 2) \
        .set("spark.executor.cores", 1).set("spark.ddl.prestartExecutors", "true").set("spark.ddl.device", "cpu")
    sc = SparkContext(conf=conf)
    try:
        assert len(E._POOLS) == 1
        pool = next(iter(E._POOLS.values()))
        pool.wait_ready()
        assert pool.world == 2 and all(p.poll() is None for p in pool.procs)
    finally:
        sc.stop()
    assert not E._POOLS


def test_elastic_resume_restores_each_workers_state(spark, tmp_path, monkeypatch):
    """EASGD workers hold state that differs per rank (own weights, own Adam slots, the center):
    a run killed on rank 1 and resumed from the per-rank checkpoint files ends bit-identical to
    an uninterrupted run (before per-rank files every rank resumed from rank 0's state)."""
    from distributeddeeplearningspark_amd.trainers import EASGD
    from distributeddeeplearningspark_amd.utils.checkpoint import latest_checkpoint

    df = _mnist_df(spark).repartition(2)

    def train(ckdir, fault):
        if fault:
            monkeypatch.setenv("DDL_FAULT_RANK", "1")
            monkeypatch.setenv("DDL_FAULT_STEP", "7")
        else:
            monkeypatch.delenv("DDL_FAULT_RANK", raising=False)
            monkeypatch.delenv("DDL_FAULT_STEP", raising=False)
        tr = EASGD(keras_model=mnist_cnn(), worker_optimizer="adam", loss="categorical_crossentropy", num_workers=2,
                   batch_size=16, communication_window=2, num_epoch=1, features_col="x", label_col="y",
                   device="cpu", checkpoint_dir=str(ckdir), checkpoint_every=1, max_restarts=1, seed=3)
        tr.train(df)
        return tr.parameter_server.center.copy()

    clean = train(tmp_path / "clean", False)
    resumed = train(tmp_path / "faulty", True)
    np.testing.assert_array_equal(resumed, clean)
    last = latest_checkpoint(str(tmp_path / "faulty"))
    ranks = os.listdir(os.path.join(str(tmp_path / "faulty"), "ranks", os.path.basename(last)))
    assert sorted(ranks) == ["rank_00000.safetensors", "rank_00001.safetensors"]
    from safetensors.torch import load_file

    t = load_file(os.path.join(str(tmp_path / "faulty"), "ranks", os.path.basename(last), ranks[0]))
    assert t["extra.center"].numel() == t["arena.master"].numel()  # both in the canonical layout
