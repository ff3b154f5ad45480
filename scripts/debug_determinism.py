"""Repeat the (composed-path) ResNet-50 forward on identical weights/input, recording
every Conv2D / BatchNormalization / pooling output, and report the first op whose
output differs between repetitions."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributeddeeplearningspark_amd.models import ResNet50, layers as L
from distributeddeeplearningspark_amd.ops import pool as P
from distributeddeeplearningspark_amd.ops.norm import reset_workspaces

REC = []


def wrap(cls, name):
    orig = cls.call

    def call(self, x, *a, **k):
        y = orig(self, x, *a, **k)
        REC.append((f"{name}:{self.name}", x.detach().clone(), y.detach().clone()))
        return y

    cls.call = call


wrap(L.Conv2D, "conv")
wrap(L.BatchNormalization, "bn")
wrap(L.Dense, "dense")
for fn in ("max_pool2d", "global_avg_pool"):
    orig = getattr(P, fn)

    def mk(orig, fn):
        def f(x, *a, **k):
            y = orig(x, *a, **k)
            REC.append((fn, x.detach().clone(), y.detach().clone()))
            return y
        return f

    setattr(P, fn, mk(orig, fn))
import distributeddeeplearningspark_amd.models.resnet as R

R.pool_ops = P

os.environ["DDL_FUSED_BLOCKS"] = "0"
torch.manual_seed(1)
x = torch.randn(8, 64, 64, 3)
y = torch.randint(0, 10, (8,))
m = ResNet50(input_shape=(64, 64, 3), num_classes=10)
m.compile("sgd", "sparse_categorical_crossentropy")
m.place("cuda:0", seed=5)
xi, yi = m.to_input(x), m.to_target(y)
runs = []
for r in range(3):
    REC.clear()
    reset_workspaces(m.device)
    with torch.no_grad():
        loss = float(m.compute_loss(xi, yi, training=True))
    torch.cuda.synchronize()
    runs.append((loss, list(REC)))
    print("run", r, "loss", loss, "ops", len(REC), flush=True)
base = runs[0][1]
for r in (1, 2):
    for i, ((n0, x0, y0), (n1, x1, y1)) in enumerate(zip(base, runs[r][1])):
        same_in = torch.equal(x0, x1)
        same_out = torch.equal(y0, y1)
        if not same_out:
            d = (y0.float() - y1.float()).abs()
            print(f"run {r}: first diff at op {i} {n0} shape={tuple(y0.shape)} same_input={same_in} "
                  f"maxdiff={d.max().item():.4g} frac_diff={(d > 0).float().mean().item():.4g} "
                  f"nan0={torch.isnan(y0).any().item()} nan1={torch.isnan(y1).any().item()}", flush=True)
            if same_in:
                bad = (d > 0).nonzero()
                print("   first differing idx", bad[:8].tolist(), flush=True)
            break
    else:
        print(f"run {r}: all op outputs identical", flush=True)
