"""Diagnose the inner fused BN-reduce: loss of consecutive backward_steps (no optimizer) per variant.

A step-to-step drift in the loss means something the backward writes persists into the next forward."""
import sys

import torch

sys.path.insert(0, ".")
from distributeddeeplearningspark_amd.models.resnet import ResNet  # noqa: E402
from distributeddeeplearningspark_amd.ops import fused_blocks as FB  # noqa: E402

DEV = "cuda:0"
torch.manual_seed(4)
x = torch.randn(64, 64, 64, 3)
y = torch.randint(0, 10, (64,))
res = {}
for fuse in (True, False, True):
    FB._FUSE_BNR_INNER = fuse
    m = ResNet(blocks=(2, 2), input_shape=(64, 64, 3), num_classes=10)
    m.compile("sgd", "sparse_categorical_crossentropy")
    m.place(DEV, seed=5)
    xd, yd = m.to_input(x), m.to_target(y)
    losses = []
    for _ in range(4):
        losses.append(float(m.backward_step(xd, yd).detach()))
    torch.cuda.synchronize()
    g = m.arena.grad.float().cpu().clone()
    print("fuse", fuse, "losses", ["%.7f" % v for v in losses], "gnorm %.6f" % g.norm().item(), flush=True)
    res.setdefault(fuse, []).append(g)
g1, g0 = res[True][0], res[False][0]
print("rel grad diff fused vs unfused %.3e" % ((g1 - g0).norm() / g0.norm()).item())
print("rel grad diff fused vs fused   %.3e" % ((res[True][1] - g1).norm() / g1.norm()).item())
