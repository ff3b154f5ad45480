"""VGG-16 (CIFAR shape, batch 256) step-time jitter: per-step GPU time (HIP events around each step)
and host issue time over 200 steps, as percentiles — separates a slow GPU (every step long) from
host stalls (host issue time spikes) and from per-step outliers."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench as B
from distributeddeeplearningspark_amd.data.ingest import SyntheticImageStream
from distributeddeeplearningspark_amd.models.optimizers import SGD
from distributeddeeplearningspark_amd.models.zoo import vgg16
from distributeddeeplearningspark_amd.parallel import comm


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    pg = comm.init_from_env(prefer_gpu=True)
    dev = pg.device
    args = type("A", (), {"reduce_dtype": None, "bucket_mb": None, "no_overlap": False, "graph": None})()
    model = vgg16(nb_classes=10, input_shape=(32, 32, 3))
    model.compile(SGD(lr=0.01, momentum=0.9, weight_decay=5e-5), "sparse_categorical_crossentropy")
    model.place(dev, seed=0)
    ddp = B.make_ddp(model, pg, args)
    stream = SyntheticImageStream(256, 32, 10, device=dev, seed=0, n_buffers=4)
    step_fn = B.make_step(ddp, args)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for _ in range(10):
        step_fn(*stream.next())
    torch.cuda.synchronize()
    host = []
    t_all = time.perf_counter()
    for i in range(steps):
        t0 = time.perf_counter()
        ev[i][0].record()
        step_fn(*stream.next())
        ev[i][1].record()
        host.append((time.perf_counter() - t0) * 1e3)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t_all) * 1e3 / steps
    gpu = [a.elapsed_time(b) for a, b in ev]

    def pct(v):
        s = sorted(v)
        return {p: round(s[min(len(s) - 1, int(p / 100 * len(s)))], 3) for p in (5, 25, 50, 75, 95, 99)}

    print(json.dumps({"steps": steps, "wall_ms_per_step": round(wall, 3), "gpu_ms": pct(gpu), "host_ms": pct(host),
                      "gpu_mean": round(statistics.mean(gpu), 3), "host_mean": round(statistics.mean(host), 3)}))


if __name__ == "__main__":
    main()
