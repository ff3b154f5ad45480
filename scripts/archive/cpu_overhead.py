"""Host-side cost of one training step: cProfile of N eager steps of --model (vgg16 / resnet50 /
bert) on the GPU, top functions by own time, plus the host time per step measured with the
GPU kept busy (no sync inside the loop) vs the GPU time per step."""
import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="vgg16", choices=["vgg16", "resnet50"])
    ap.add_argument("--steps", type=int, default=30)
    args = ap.parse_args()
    from distributeddeeplearningspark_amd.data.ingest import SyntheticImageStream
    from distributeddeeplearningspark_amd.models import ResNet50
    from distributeddeeplearningspark_amd.models.optimizers import SGD
    from distributeddeeplearningspark_amd.models.zoo import vgg16
    from distributeddeeplearningspark_amd.parallel.comm import ProcessGroup
    from distributeddeeplearningspark_amd.parallel.ddp import DataParallel

    img, ncls = (32, 10) if args.model == "vgg16" else (224, 1000)
    m = vgg16(nb_classes=ncls, input_shape=(img, img, 3)) if args.model == "vgg16" else ResNet50(
        input_shape=(img, img, 3), num_classes=ncls)
    m.compile(SGD(lr=0.01, momentum=0.9, weight_decay=5e-5), "sparse_categorical_crossentropy")
    dev = torch.device("cuda:0")
    m.place(dev, seed=0)
    ddp = DataParallel(m, ProcessGroup(0, 1, 0, dev, None))
    stream = SyntheticImageStream(256, img, ncls, device=dev, seed=0, n_buffers=4)
    batches = [stream.next() for _ in range(4)]
    for i in range(5):
        ddp.train_step(*batches[i % 4])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for i in range(args.steps):
        ddp.train_step(*batches[i % 4])
    t_issue = time.perf_counter() - t0
    e1.record()
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    print(f"host issue {t_issue / args.steps * 1e3:.3f} ms/step, wall {t_all / args.steps * 1e3:.3f} ms/step, "
          f"GPU {e0.elapsed_time(e1) / args.steps:.3f} ms/step", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for i in range(args.steps):
        ddp.train_step(*batches[i % 4])
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(45)
    st.sort_stats("cumulative").print_stats(45)


if __name__ == "__main__":
    main()
