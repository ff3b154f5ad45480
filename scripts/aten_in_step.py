"""Which ATen (non-ddl) GPU kernels a ResNet-50 training step still launches, and from where.

torch.profiler over one warm bench step (forward, backward, SGD) with Python stacks; prints every aten op
that launched a GPU kernel, with its count and the innermost framework frame that called it."""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from torch.profiler import ProfilerActivity, profile

from distributeddeeplearningspark_amd.models import ResNet50
from distributeddeeplearningspark_amd.models.optimizers import SGD

dev = torch.device("cuda", 0)
model = ResNet50(input_shape=(224, 224, 3), num_classes=1000)
model.compile(SGD(lr=0.1, momentum=0.9, weight_decay=5e-5), "sparse_categorical_crossentropy")
model.place(dev, seed=0)
x = torch.randint(0, 256, (256, 224, 224, 3), dtype=torch.uint8, device=dev)
y = torch.randint(0, 1000, (256,), device=dev)
for _ in range(3):
    model.train_on_batch(x, y)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    model.train_on_batch(x, y)
    torch.cuda.synchronize()

sites = collections.Counter()
for e in prof.events():
    if not e.name.startswith("aten::") or e.device_type != torch.autograd.DeviceType.CPU:
        continue
    if not e.kernels:  # no GPU kernel launched by this op
        continue
    frame = next((f for f in (e.stack or []) if "distributeddeeplearningspark_amd" in f), "?")
    sites[(e.name, frame)] += 1
for (name, frame), n in sites.most_common(40):
    print(f"{n:4d}  {name:28s} {frame}")
