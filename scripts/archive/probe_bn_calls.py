"""Which BatchNorm sweeps a ResNet-50 training step still launches, with their shapes.

Wraps the native BN entry points (bn_bwd_reduce / bn_bwd_dx / bn_apply / finalizes) with a counting
proxy, runs warm steps of the bench model, and prints one line per call site of the last step:
entry point, rows x channels, mode.  Used to find the reduce sweeps the fused epilogues do not cover."""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributeddeeplearningspark_amd.ops import _native, fused_blocks, norm

calls = []
_real = _native.C


class _Proxy:
    def __init__(self, mod):
        self._m = mod

    def __getattr__(self, name):
        f = getattr(self._m, name)
        if name.startswith("bn_") or name in ("splitk_finalize", "filter_taps_transpose", "transpose_bf16",
                                               "wgrad_slab_reduce"):
            def w(*a, **k):
                shp = [tuple(x.shape) for x in a if isinstance(x, torch.Tensor)][:3]
                ints = [x for x in a if isinstance(x, int)]
                calls.append((name, shp, ints))
                return f(*a, **k)
            return w
        return f


def C():
    return _Proxy(_real())


fused_blocks.C = C
norm.C = C

from distributeddeeplearningspark_amd.models import ResNet50  # noqa: E402
from distributeddeeplearningspark_amd.models.optimizers import SGD  # noqa: E402

dev = torch.device("cuda", 0)
model = ResNet50(input_shape=(224, 224, 3), num_classes=1000)
model.compile(SGD(lr=0.1, momentum=0.9, weight_decay=5e-5), "sparse_categorical_crossentropy")
model.place(dev, seed=0)
x = torch.randint(0, 256, (256, 224, 224, 3), dtype=torch.uint8, device=dev)
y = torch.randint(0, 1000, (256,), device=dev)
for i in range(3):
    calls.clear()
    model.train_on_batch(x, y)
torch.cuda.synchronize()
cnt = collections.Counter(c[0] for c in calls)
print("per step:", dict(cnt))
for c in calls:
    if c[0] in ("bn_bwd_reduce",):
        print(c)
