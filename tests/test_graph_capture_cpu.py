"""models/step.py:graph_capture: the cyclic garbage collector is off for the whole capture (a collection inside
a capture runs HIP-illegal destructors) and its previous state is restored, also when the capture raises."""
import contextlib
import gc

import pytest
import torch


def test_graph_capture_disables_gc_and_restores(monkeypatch):
    from distributeddeeplearningspark_amd.models import step

    seen = []

    @contextlib.contextmanager
    def fake_graph(g, stream=None):
        seen.append(gc.isenabled())
        yield

    monkeypatch.setattr(torch.cuda, "graph", fake_graph)
    assert gc.isenabled()
    with step.graph_capture(object(), None):
        seen.append(gc.isenabled())
    assert seen == [False, False] and gc.isenabled()
    with pytest.raises(RuntimeError):
        with step.graph_capture(object(), None):
            raise RuntimeError("capture failed")
    assert gc.isenabled()
    gc.disable()
    try:
        with step.graph_capture(object(), None):
            pass
        assert not gc.isenabled()  # a caller that had it off keeps it off
    finally:
        gc.enable()
