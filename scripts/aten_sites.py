"""Where do the remaining ATen (non-ddl) GPU ops of a training step come from?  Runs a few
steps of --model under torch.profiler with Python stacks and prints, per ATen op that
launches device work, its call count per step and the innermost framework frames."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from torch.profiler import ProfilerActivity, profile

OPS = ("aten::fill_", "aten::zero_", "aten::copy_", "aten::add_", "aten::constant_pad_nd", "aten::sum",
       "aten::mul_", "aten::zeros", "aten::cat", "aten::index_select", "aten::where", "aten::sub")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="vgg16", choices=["vgg16", "resnet50"])
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    from distributeddeeplearningspark_amd.data.ingest import SyntheticImageStream
    from distributeddeeplearningspark_amd.models import ResNet50
    from distributeddeeplearningspark_amd.models.optimizers import SGD
    from distributeddeeplearningspark_amd.models.zoo import vgg16

    img, ncls = (32, 10) if args.model == "vgg16" else (224, 1000)
    m = vgg16(nb_classes=ncls, input_shape=(img, img, 3)) if args.model == "vgg16" else ResNet50(
        input_shape=(img, img, 3), num_classes=ncls)
    m.compile(SGD(lr=0.01, momentum=0.9, weight_decay=5e-5), "sparse_categorical_crossentropy")
    m.place("cuda:0", seed=0)
    stream = SyntheticImageStream(256, img, ncls, device=torch.device("cuda:0"), seed=0, n_buffers=2)
    for _ in range(3):
        x, y = stream.next()
        m.train_on_batch(x, y)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for _ in range(args.steps):
            x, y = stream.next()
            m.train_on_batch(x, y)
        torch.cuda.synchronize()
    seen = {}
    for ev in prof.events():
        if ev.name not in OPS:
            continue
        frames = [f for f in (ev.stack or []) if "distributeddeeplearningspark_amd" in f or "scripts/" in f]
        key = (ev.name, " <- ".join(f.split("distributeddeeplearningspark_amd/")[-1] for f in frames[:3]))
        seen[key] = seen.get(key, 0) + 1
    for (name, where), n in sorted(seen.items(), key=lambda kv: -kv[1]):
        print(f"{n / args.steps:6.1f}/step  {name:24s} {where}")


if __name__ == "__main__":
    main()
