"""One MNIST replica (batch 16) stepping through a captured 5-step window, alone on the GPU:
ms per step, for the launch-diet / kernel work on the co-located workers (examples/ddl_mnist.py)."""
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import torch

from distributeddeeplearningspark_amd.models.zoo import mnist_cnn
from distributeddeeplearningspark_amd.ops._native import C

m = mnist_cnn()
m.compile("adam", "categorical_crossentropy")
m.place("cuda", seed=0)
X = torch.rand(7500, 28, 28, 1, device="cuda").to(torch.bfloat16)
Y = torch.nn.functional.one_hot(torch.randint(0, 10, (7500,), device="cuda"), 10).float()
sx, sy = torch.empty_like(X[:16]), torch.empty_like(Y[:16])
ctr = torch.zeros(1, dtype=torch.int32, device="cuda")
hist = torch.zeros(100000, device="cuda")


def step(captured, more=False):
    C().batch_fetch([X, Y], [sx, sy], ctr, 468)
    loss = m.backward_step(m.to_input(sx), m.to_target(sy))
    if captured:
        m.optimizer.captured_update(1.0, zero_grads=more)
    else:
        m.optimizer.step(1.0)
    C().step_record(loss.detach().float().reshape(1), hist, ctr)


for _ in range(3):
    step(False)
m.optimizer.enable_device_step()
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    with torch.cuda.graph(g, stream=s):
        for i in range(5):
            step(True, more=i < 4)
torch.cuda.current_stream().wait_stream(s)
for _ in range(10):
    g.replay()
torch.cuda.synchronize()
n = int(os.environ.get("REPS", "400"))
t0 = time.perf_counter()
for _ in range(n):
    g.replay()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / (5 * n) * 1e6
print(f"MNIST replica step (graph window of 5): {dt:.1f} us/step, loss {hist[int(ctr.item()) - 1].item():.4f}")
