"""Native host runtime: batch loader (csrc/runtime/loader.cpp)."""
import numpy as np
import pytest
import torch

from distributeddeeplearningspark_amd.ops._native import has_native

pytestmark = pytest.mark.skipif(not has_native(), reason="native extension not built")


def test_batch_loader_order_and_tail():
    from distributeddeeplearningspark_amd.data.ingest import ShardLoader

    x = np.arange(50 * 3, dtype=np.float32).reshape(50, 3)
    y = np.arange(50, dtype=np.int64)
    ld = ShardLoader(x, y, batch=8, drop_last=True, n_buffers=3)
    assert len(ld) == 6
    got = [(xb.clone(), yb.clone()) for xb, yb in ld]
    assert len(got) == 6
    for b, (xb, yb) in enumerate(got):
        np.testing.assert_array_equal(xb.numpy(), x[b * 8:(b + 1) * 8])
        np.testing.assert_array_equal(yb.numpy(), y[b * 8:(b + 1) * 8])
    ld2 = ShardLoader(x, y, batch=8, drop_last=False)
    sizes = [xb.shape[0] for xb, _ in ld2]
    assert sizes == [8] * 6 + [2]


def test_batch_loader_shuffle_is_permutation_per_epoch():
    from distributeddeeplearningspark_amd.data.ingest import ShardLoader

    x = np.arange(64, dtype=np.float32).reshape(64, 1)
    ld = ShardLoader(x, None, batch=16, shuffle=True, seed=3, n_buffers=2)
    e0 = torch.cat([xb.clone() for xb, _ in ld]).flatten().numpy()
    e1 = torch.cat([xb.clone() for xb, _ in ld]).flatten().numpy()
    assert sorted(e0.tolist()) == list(range(64)) and sorted(e1.tolist()) == list(range(64))
    assert not np.array_equal(e0, e1) and not np.array_equal(e0, np.arange(64))


def test_batch_loader_large_rows_multithreaded():
    from distributeddeeplearningspark_amd.data.ingest import ShardLoader

    x = np.random.default_rng(0).integers(0, 255, size=(96, 128, 128, 3), dtype=np.uint8)  # > 8 MB per batch of 48
    ld = ShardLoader(x, None, batch=48, shuffle=True, seed=1, threads=4)
    rows = torch.cat([xb.clone() for xb, _ in ld]).numpy()
    assert rows.shape == x.shape
    key = lambda a: a.reshape(a.shape[0], -1)[:, :16].tobytes()  # noqa: E731
    assert sorted(key(r[None]) for r in rows) == sorted(key(r[None]) for r in x)
