"""Where do the remaining ATen (non-ddl) GPU ops of a training step come from?  Wraps the torch
entry points that launch small device kernels (fills, copies, pads, reductions, casts) and
counts, per framework call site, how often one step calls them on a CUDA tensor."""
import argparse
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

COUNTS = collections.Counter()
ACTIVE = [False]


def _site():
    for fr in reversed(traceback.extract_stack()[:-2]):
        if "distributeddeeplearningspark_amd" in fr.filename or fr.filename.endswith("bench.py"):
            return f"{fr.filename.split('distributeddeeplearningspark_amd/')[-1]}:{fr.lineno} {fr.line}"
    return "?"


def _wrap(owner, name, is_cuda):
    orig = getattr(owner, name)

    def f(*a, **k):
        if ACTIVE[0] and is_cuda(a, k):
            COUNTS[(name, _site())] += 1
        return orig(*a, **k)

    setattr(owner, name, f)


def _first_cuda(a, k):
    return any(isinstance(x, torch.Tensor) and x.is_cuda for x in list(a) + list(k.values()))


def _dev_kw(a, k):
    d = k.get("device")
    return d is not None and torch.device(d).type == "cuda"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="vgg16", choices=["vgg16", "resnet50"])
    args = ap.parse_args()
    from distributeddeeplearningspark_amd.data.ingest import SyntheticImageStream
    from distributeddeeplearningspark_amd.models import ResNet50
    from distributeddeeplearningspark_amd.models.optimizers import SGD
    from distributeddeeplearningspark_amd.models.zoo import vgg16
    from distributeddeeplearningspark_amd.parallel.comm import ProcessGroup
    from distributeddeeplearningspark_amd.parallel.ddp import DataParallel

    for n in ("zero_", "fill_", "copy_", "to", "sum", "add_", "mul_", "div_", "clamp_min", "float", "contiguous",
              "__mul__", "__truediv__", "__ne__", "mean", "index_select", "clone"):
        _wrap(torch.Tensor, n, _first_cuda)
    for n in ("zeros", "zeros_like", "ones", "full", "empty_like", "where", "cat", "stack"):
        _wrap(torch, n, lambda a, k: _first_cuda(a, k) or _dev_kw(a, k))
    _wrap(F, "pad", _first_cuda)

    img, ncls = (32, 10) if args.model == "vgg16" else (224, 1000)
    m = vgg16(nb_classes=ncls, input_shape=(img, img, 3)) if args.model == "vgg16" else ResNet50(
        input_shape=(img, img, 3), num_classes=ncls)
    m.compile(SGD(lr=0.01, momentum=0.9, weight_decay=5e-5), "sparse_categorical_crossentropy")
    dev = torch.device("cuda:0")
    m.place(dev, seed=0)
    ddp = DataParallel(m, ProcessGroup(0, 1, 0, dev, None))
    stream = SyntheticImageStream(256, img, ncls, device=dev, seed=0, n_buffers=2)
    for _ in range(3):
        ddp.train_step(*stream.next())
    torch.cuda.synchronize()
    ACTIVE[0] = True
    ddp.train_step(*stream.next())
    ACTIVE[0] = False
    torch.cuda.synchronize()
    for (name, where), n in sorted(COUNTS.items(), key=lambda kv: -kv[1]):
        print(f"{n:4d}  {name:14s} {where}")


if __name__ == "__main__":
    main()
