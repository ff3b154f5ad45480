"""Co-located dist-keras workers on ONE MI355X (DDL_WORKERS_PER_GPU).

Default: the workers run as in-process replica groups (parallel/replicas.py: graph-replayed
windows on one HIP stream per replica, one commit kernel over all replicas).  With
DDL_REPLICA_GROUPS=0 they are separate processes whose commits go through the device-side IPC
exchange (parallel/colocated.py) or, with DDL_COLOCATED_EXCHANGE=0, the host-staged gloo path.
All three must give the same center (one summation order), the same update law and the same
per-worker loss histories for ADAG, DynSGD and EASGD."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _frame(n=512, seed=0):
    from distributeddeeplearningspark_amd.sql.dataframe import from_columns

    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 16)).astype(np.float32)
    y = (X @ rng.normal(size=(16, 1))).astype(np.float32)
    return from_columns({"features": X, "label": y}, num_partitions=4)


def _model():
    from distributeddeeplearningspark_amd.models import Dense, Sequential

    m = Sequential([Dense(32, input_shape=(16,), activation="relu"), Dense(1)])
    m.compile("adam", "mean_squared_error")
    return m


def _train(algo, exchange, monkeypatch, groups="0"):
    from distributeddeeplearningspark_amd import trainers as T
    from distributeddeeplearningspark_amd.parallel.executors import shutdown_all

    monkeypatch.setenv("DDL_WORKERS_PER_GPU", "4")
    monkeypatch.setenv("DDL_REPLICA_GROUPS", groups)
    monkeypatch.setenv("DDL_COLOCATED_EXCHANGE", "1" if exchange else "0")
    cls = {"adag": T.ADAG, "dynsgd": T.DynSGD, "easgd": T.EASGD}[algo]
    kw = dict(keras_model=_model(), worker_optimizer="adam", loss="mean_squared_error", num_workers=4,
              batch_size=16, num_epoch=2, features_col="features", label_col="label")
    if algo != "easgd":
        kw["communication_window"] = 2
    tr = cls(**kw)
    m = tr.train(_frame())
    res = tr._results
    shutdown_all()
    return m.arena.master.detach().cpu().clone(), tr.parameter_server.num_updates, res


@pytest.mark.parametrize("algo", ["adag", "dynsgd", "easgd"])
def test_colocated_exchange_matches_host_staged(algo, monkeypatch):
    w_dev, n_dev, res_dev = _train(algo, True, monkeypatch)
    w_host, n_host, res_host = _train(algo, False, monkeypatch)
    assert n_dev == n_host
    assert all(r["commit_wait_s"] is not None for r in res_dev), "device exchange was not used"
    assert all(r["commit_wait_s"] is None for r in res_host)
    torch.testing.assert_close(w_dev, w_host, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("algo", ["adag", "dynsgd", "easgd"])
def test_replica_group_matches_process_workers(algo, monkeypatch):
    w_grp, n_grp, res_grp = _train(algo, True, monkeypatch, groups="1")
    w_ipc, n_ipc, res_ipc = _train(algo, True, monkeypatch, groups="0")
    assert n_grp == n_ipc
    assert all(r.get("replica_group", {}).get("replicas") == 4 for r in res_grp), "replica group not used"
    assert all(r["graph"] for r in res_grp), "replica windows were not graph-replayed"
    assert all(r["commit_wait_s"] is not None for r in res_ipc)
    torch.testing.assert_close(w_grp, w_ipc, rtol=1e-4, atol=1e-5)
    for a, b in zip(res_grp, res_ipc):
        assert len(a["history"]) == len(b["history"])
        np.testing.assert_allclose(a["history"], b["history"], rtol=1e-3, atol=1e-5)
