"""Dropout inside a graph-replayed step (models/step.py + ops/act.py dropout_step_counter): the capture-time seeds
are mixed with a device step counter that the captured step ticks, so every replay draws a fresh mask (a frozen
mask would repeat the same loss on the same batch at lr = 0), and the forward and backward of one replay share
their mask (the gradient of the dropped units is zero)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _model(lr):
    from distributeddeeplearningspark_amd.models import Dense, Dropout, Sequential
    from distributeddeeplearningspark_amd.models.optimizers import SGD

    m = Sequential([Dense(256, input_shape=(64,), activation="relu"), Dropout(0.5), Dense(10, activation="softmax")])
    m.compile(SGD(lr=lr), "sparse_categorical_crossentropy")
    m.place("cuda:0", seed=0)
    return m


def test_graph_replay_draws_fresh_dropout_masks():
    from distributeddeeplearningspark_amd.models.step import CompiledTrainStep
    from distributeddeeplearningspark_amd.ops.act import dropout_step_counter

    m = _model(0.0)
    assert m.graph_capturable
    g = torch.Generator().manual_seed(0)
    x = m.to_input(torch.randn(128, 64, generator=g))
    y = m.to_target(torch.randint(0, 10, (128,), generator=g))
    step = CompiledTrainStep(m, warmup=2)
    c0 = float(dropout_step_counter("cuda:0"))
    losses = [float(step(x, y)) for _ in range(7)]
    assert step.captured, step.fallback_reason
    assert float(dropout_step_counter("cuda:0")) == c0 + 5  # one tick per replay
    replayed = losses[2:]
    assert len(set(replayed)) == len(replayed), replayed  # lr = 0: only the masks change the loss


def test_graph_replayed_dropout_trains():
    from distributeddeeplearningspark_amd.models.step import CompiledTrainStep

    m = _model(0.1)
    g = torch.Generator().manual_seed(1)
    w = torch.randn(64, 10, generator=g)
    x = torch.randn(512, 64, generator=g)
    y = (x @ w).argmax(1)
    xs, ys = m.to_input(x), m.to_target(y)
    step = CompiledTrainStep(m, warmup=2)
    losses = [float(step(xs, ys)) for _ in range(200)]
    assert step.captured
    assert sum(losses[-20:]) / 20 < 0.5 * sum(losses[:20]) / 20, (losses[:5], losses[-5:])
