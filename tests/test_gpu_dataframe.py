"""DataFrame-fed training on the GPU: a uint8 image frame through SynchronousDataParallel with
the shard resident in HBM vs streamed through the native pinned ring (ShardLoader), and the
partition predictor on the GPU path."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _frame(n=192, hw=16, seed=0):
    from distributeddeeplearningspark_amd.sql.dataframe import from_columns

    rng = np.random.default_rng(seed)
    imgs = rng.integers(0, 256, (n, hw, hw, 3), dtype=np.uint8)
    labels = rng.integers(0, 10, n)
    return from_columns({"features": imgs, "label": labels}, num_partitions=1), imgs, labels


def _model(hw=16):
    from distributeddeeplearningspark_amd.models import Activation, Conv2D, Dense, Flatten, Sequential

    m = Sequential([Conv2D(16, (3, 3), input_shape=(hw, hw, 3)), Activation("relu"), Flatten(),
                    Dense(10, activation="softmax")])
    m.compile("sgd", "sparse_categorical_crossentropy")
    m.input_mean, m.input_std = (0.0, 0.0, 0.0), (255.0, 255.0, 255.0)  # uint8 pixels -> [0, 1] on the device
    return m


@pytest.mark.parametrize("ingest", ["resident", "stream"])
def test_syncdp_trains_from_uint8_frame(ingest):
    from distributeddeeplearningspark_amd.trainers import SynchronousDataParallel

    df, imgs, labels = _frame()
    results = {}
    for mode in ("resident", ingest):
        torch.manual_seed(0)
        m = _model()
        tr = SynchronousDataParallel(m, worker_optimizer="sgd", loss="sparse_categorical_crossentropy",
                                     num_workers=1, batch_size=32, num_epoch=2, features_col="features",
                                     label_col="label", ingest=mode, seed=0)
        trained = tr.train(df)
        assert tr._results[0]["ingest"] == mode
        assert tr.parameter_server.num_updates == 2 * (192 // 32)
        results[mode] = (trained.arena.master.detach().cpu().clone(), tr.history[0])
    w_res, h_res = results["resident"]
    w_mode, h_mode = results[ingest]
    assert len(h_mode) == 12 and np.isfinite(h_mode).all()
    # same batches in the same order: only split-K atomic summation order may differ
    torch.testing.assert_close(w_mode, w_res, rtol=2e-3, atol=2e-4)


def test_gpu_predictor_on_uint8_frame():
    from distributeddeeplearningspark_amd.predictors import ModelPredictor

    df, imgs, _ = _frame(n=70)
    m = _model()
    m.place("cuda:0", seed=1)
    out = ModelPredictor(m, device="cuda:0", batch_size=32).predict(df)
    p = np.stack([r["prediction"].toArray() for r in out.collect()])
    assert p.shape == (70, 10)
    np.testing.assert_allclose(p.sum(1), 1.0, atol=2e-2)  # bf16 softmax rows
    ref = m.predict(imgs, batch_size=70)
    np.testing.assert_allclose(p, ref, atol=1e-3)


def test_shard_loader_host_runs_ahead_of_copies():
    """The streaming loader hands out batches while their H2D copies are still in flight: the
    compute stream is kept busy so the host runs several batches ahead, and every batch must
    still equal the resident slice (the slot is reused only after its copy event completed, and
    the batch tensors are recorded on the compute stream)."""
    from distributeddeeplearningspark_amd.data.ingest import ShardLoader

    rng = np.random.default_rng(3)
    X = rng.integers(0, 256, (40 * 64, 96, 96, 3), dtype=np.uint8)  # 27 KB rows, 1.7 MB per batch
    Y = np.arange(X.shape[0], dtype=np.int64)
    loader = ShardLoader(X, Y, 64, device="cuda:0", n_buffers=4)
    busy = torch.randn(2048, 2048, device="cuda:0")
    sums = []
    for xd, yd in loader:
        for _ in range(3):  # keep the compute stream behind the host
            busy = busy @ busy
            busy = busy / busy.norm()
        sums.append((xd.to(torch.int64).sum(dim=(1, 2, 3)), yd.clone()))
    torch.cuda.synchronize()
    assert len(sums) == 40
    for b, (s, yd) in enumerate(sums):
        ref = torch.from_numpy(X[b * 64:(b + 1) * 64].astype(np.int64).sum(axis=(1, 2, 3)))
        assert torch.equal(s.cpu(), ref), b
        assert torch.equal(yd.cpu(), torch.from_numpy(Y[b * 64:(b + 1) * 64]))
