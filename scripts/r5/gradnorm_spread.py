"""Gradient-norm spread of the small ResNet-50 step (tests/test_gpu_kernels.py): fp32 CPU unperturbed and
under 2^-9 / 2^-7 relative input perturbations, the HIP bf16 path (two runs), the HIP path in
deterministic mode, and the same bf16 model through PyTorch ops (DDL_BACKEND=torch).  Is the HIP path's
~4 % lower norm a bias of the HIP kernels, of bf16 itself, or the spread of a chaotic network?"""
import os
import sys

sys.path.insert(0, os.getcwd())
import torch

from distributeddeeplearningspark_amd.models import ResNet50

torch.manual_seed(0)
x = torch.randn(16, 64, 64, 3)
y = torch.randint(0, 10, (16,))


def run(dev, xin, backend=None, det=False):
    old = os.environ.get("DDL_BACKEND")
    if backend:
        os.environ["DDL_BACKEND"] = backend
    from distributeddeeplearningspark_amd.ops import determinism as D
    try:
        m = ResNet50(input_shape=(64, 64, 3), num_classes=10)
        m.compile("sgd", "sparse_categorical_crossentropy")
        m.place(dev, seed=3)
        if det:
            D.set_enabled(True)
        loss = m.backward_step(m.to_input(xin), m.to_target(y))
        return float(loss.detach()), m.arena.grad.float().norm().item()
    finally:
        if det:
            D.set_enabled(False)
        if backend:
            if old is None:
                os.environ.pop("DDL_BACKEND", None)
            else:
                os.environ["DDL_BACKEND"] = old


print("cpu fp32", run("cpu", x), flush=True)
for k, s in enumerate((2.0 ** -9, 2.0 ** -9, 2.0 ** -9, 2.0 ** -7, 2.0 ** -7)):
    g = torch.Generator().manual_seed(100 + k)
    xp = x * (1 + s * torch.randn(x.shape, generator=g))
    print(f"cpu fp32 input x(1+{s:g} n) seed {k}", run("cpu", xp), flush=True)
print("hip bf16 run 1", run("cuda", x), flush=True)
print("hip bf16 run 2", run("cuda", x), flush=True)
try:
    print("hip bf16 deterministic", run("cuda", x, det=True), flush=True)
except Exception as e:
    print("deterministic mode:", type(e).__name__, e)
print("torch bf16 (DDL_BACKEND=torch)", run("cuda", x, backend="torch"), flush=True)
for k in range(3):
    g = torch.Generator().manual_seed(200 + k)
    xp = x * (1 + 2.0 ** -9 * torch.randn(x.shape, generator=g))
    print(f"hip bf16 input x(1+2^-9 n) seed {k}", run("cuda", xp), flush=True)
