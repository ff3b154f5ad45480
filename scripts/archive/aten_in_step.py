"""Which ATen GPU ops a ResNet-50 bench step (DataParallel.train_step, as bench.py runs it) still issues, and
from where: torch.zeros / zeros_like / Tensor.zero_ / fill_ / copy_ / clone / contiguous are wrapped during one
warm step and every call on a CUDA tensor is counted by its innermost framework call site."""
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributeddeeplearningspark_amd.data.ingest import SyntheticImageStream
from distributeddeeplearningspark_amd.models import ResNet50
from distributeddeeplearningspark_amd.models.optimizers import SGD
from distributeddeeplearningspark_amd.parallel import comm
from distributeddeeplearningspark_amd.parallel.ddp import DataParallel

pg = comm.init_from_env(prefer_gpu=True)
dev = pg.device
model = ResNet50(input_shape=(224, 224, 3), num_classes=1000)
model.compile(SGD(lr=0.1, momentum=0.9, weight_decay=5e-5), "sparse_categorical_crossentropy")
model.place(dev, seed=0)
ddp = DataParallel(model, pg)
stream = SyntheticImageStream(256, 224, 1000, device=dev, seed=0, n_buffers=4)
for _ in range(3):
    ddp.train_step(*stream.next())
torch.cuda.synchronize()

sites = collections.Counter()
active = [False]


def site():
    for fr in reversed(traceback.extract_stack()[:-2]):
        if "distributeddeeplearningspark_amd" in fr.filename:
            return f"{os.path.relpath(fr.filename, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))}:{fr.lineno}"
    return "?"


def wrap(owner, name, is_cuda):
    orig = getattr(owner, name)

    def w(*a, **k):
        r = orig(*a, **k)
        if active[0]:
            try:
                if is_cuda(a, k, r):
                    sites[(name, site())] += 1
            except Exception:
                pass
        return r
    setattr(owner, name, w)


def out_cuda(a, k, r):
    return isinstance(r, torch.Tensor) and r.is_cuda


for nm in ("zeros", "zeros_like", "ones", "full", "cat", "stack"):
    wrap(torch, nm, out_cuda)
for nm in ("zero_", "fill_", "copy_", "clone", "contiguous", "add_", "mul_", "to"):
    wrap(torch.Tensor, nm, lambda a, k, r, nm=nm: isinstance(a[0], torch.Tensor) and a[0].is_cuda
         and r is not a[0] if nm in ("contiguous", "to") else isinstance(a[0], torch.Tensor) and a[0].is_cuda)

active[0] = True
ddp.train_step(*stream.next())
torch.cuda.synchronize()
active[0] = False
for (name, where), n in sites.most_common(40):
    print(f"{n:4d}  {name:12s} {where}")
