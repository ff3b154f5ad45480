"""Bisect which part of a training step breaks hipGraph capture (debug aid)."""
import sys
import traceback

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from distributeddeeplearningspark_amd.models import zoo  # noqa: E402


def try_capture(name, fn):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    try:
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                fn()
        torch.cuda.current_stream().wait_stream(s)
        g.replay()
        torch.cuda.synchronize()
        print(f"[ok]   {name}", flush=True)
    except Exception:
        print(f"[FAIL] {name}\n{traceback.format_exc()[-1500:]}", flush=True)
        torch.cuda.synchronize()


m = zoo.mnist_cnn()
m.compile("adam", "categorical_crossentropy")
m.place("cuda:0")
x = m.to_input(torch.rand(16, 28, 28, 1))
y = m.to_target(torch.nn.functional.one_hot(torch.randint(0, 10, (16,)), 10).float())
for _ in range(2):
    m.train_on_batch(x, y)
torch.cuda.synchronize()
L = m.layers if hasattr(m, "layers") else m.sublayers()
h = x
for i, layer in enumerate(L):
    hh = h
    try_capture(f"fwd layer {i} {type(layer).__name__}", lambda: layer(hh, training=True))
    with torch.no_grad():
        h = layer(h, training=True)
try_capture("forward", lambda: m.forward(x, training=True))
try_capture("loss", lambda: m.compute_loss(x, y))
try_capture("backward_step", lambda: m.backward_step(x, y))
m.optimizer.enable_device_step()
try_capture("optimizer", lambda: m.optimizer._apply(m.arena.master, m.arena.grad, m.arena.compute, 1.0))
