"""Call sites of the ATen fills / copies inside one ResNet-50 (MODEL=vgg16: VGG-16 CIFAR-shape) training step
(bench.py's DataParallel step, batch 256): torch.zeros / zeros_like / full / Tensor.zero_ / fill_ / copy_ / clone on CUDA tensors are
wrapped and counted by the package frame that called them."""
import collections
import os
import sys
import traceback

sys.path.insert(0, os.getcwd())
import torch

from distributeddeeplearningspark_amd.models import ResNet50
from distributeddeeplearningspark_amd.models.optimizers import SGD
from distributeddeeplearningspark_amd.parallel import comm
from distributeddeeplearningspark_amd.parallel.ddp import DataParallel

B = int(os.environ.get("BATCH", "256"))
if os.environ.get("MODEL") == "vgg16":
    from distributeddeeplearningspark_amd.models.zoo import vgg16
    IMG, NCLS = 32, 10
    m = vgg16(nb_classes=NCLS, input_shape=(IMG, IMG, 3))
else:
    IMG, NCLS = 224, 1000
    m = ResNet50(input_shape=(IMG, IMG, 3), num_classes=NCLS)
m.compile(SGD(lr=0.1, momentum=0.9, weight_decay=5e-5), "sparse_categorical_crossentropy")
m.place("cuda:0", seed=0)  # as bench.py (LOCAL_RANK device)
x = torch.randint(0, 255, (B, IMG, IMG, 3), dtype=torch.uint8).pin_memory()
y = torch.randint(0, NCLS, (B,))
eng = DataParallel(m, comm.init_from_env(prefer_gpu=True), bucket_mb=32.0)
step = lambda: eng.train_step(m.to_input(x), m.to_target(y))
for _ in range(3):
    step()
torch.cuda.synchronize()

counts = collections.Counter()
ACTIVE = [False]


def site():
    for f in reversed(traceback.extract_stack()[:-2]):
        if "distributeddeeplearningspark_amd" in f.filename or "bench" in f.filename:
            return f"{f.filename.split('repo/')[-1]}:{f.lineno} {f.line.strip()[:70]}"
    return "?"


def wrap_fn(mod, name):
    orig = getattr(mod, name)

    def w(*a, **k):
        out = orig(*a, **k)
        if ACTIVE[0] and isinstance(out, torch.Tensor) and out.is_cuda:
            counts[f"{name} @ {site()}"] += 1
        return out
    setattr(mod, name, w)


def wrap_method(name):
    orig = getattr(torch.Tensor, name)

    def w(self, *a, **k):
        if ACTIVE[0] and self.is_cuda:
            counts[f"Tensor.{name} @ {site()}"] += 1
        return orig(self, *a, **k)
    setattr(torch.Tensor, name, w)


for n in ("zeros", "zeros_like", "full", "ones", "ones_like"):
    wrap_fn(torch, n)
for n in ("zero_", "fill_", "copy_", "clone", "add_", "contiguous"):
    wrap_method(n)
ACTIVE[0] = True
step()
torch.cuda.synchronize()
ACTIVE[0] = False
for k, v in counts.most_common():
    print(f"{v:4d}  {k}")
