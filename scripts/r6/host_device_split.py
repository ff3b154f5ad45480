"""Host dispatch time vs device time per training step (verdict r5 item 5).

For each model (VGG-16 CIFAR-shape, ResNet-50) and step form (eager launches, whole-step hipGraph replay):
  * wall_ms: synchronized wall time per step over K steps (what bench.py reports);
  * host_ms: host time to ISSUE one step while the GPU is held busy by a long sleep kernel queued first, so the
    host never waits on the device (valid only if the sleep is still running when the K steps are issued —
    checked, reported as host_valid);
  * device_ms: GPU time per step with the host out of the way: the K steps queued behind the sleep, timed by
    events from the sleep's end to the last step's end.
host_ms > device_ms means the step is host-bound (the GPU idles between launches)."""
import json
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import torch


def build(model_name, graph):
    from distributeddeeplearningspark_amd.data.ingest import SyntheticImageStream
    from distributeddeeplearningspark_amd.models import ResNet50
    from distributeddeeplearningspark_amd.models.optimizers import SGD
    from distributeddeeplearningspark_amd.models.step import CompiledTrainStep
    from distributeddeeplearningspark_amd.models.zoo import vgg16
    from distributeddeeplearningspark_amd.parallel import comm
    from distributeddeeplearningspark_amd.parallel.ddp import DataParallel

    dev = torch.device("cuda:0")
    if model_name == "bert":  # eager only (the BERT step is not graph-captured)
        from distributeddeeplearningspark_amd.data.synthetic import mlm_batch
        from distributeddeeplearningspark_amd.models.bert import BertConfig, BertForMaskedLM
        from distributeddeeplearningspark_amd.models.optimizers import AdamW

        cfg = BertConfig()
        m = BertForMaskedLM(cfg)
        m.compile(AdamW(lr=1e-4, weight_decay=0.01), "sparse_categorical_crossentropy")
        m.place(dev, seed=0)
        ddp = DataParallel(m, comm.ProcessGroup(0, 1, 0, dev, None))
        bs = [mlm_batch(32, 512, cfg.vocab_size, seed=i) for i in range(4)]
        bs = [(m.to_input(x), m.to_target(y)) for x, y in bs]
        it = [0]

        def step():
            it[0] += 1
            return ddp.train_step(*bs[it[0] % 4])
        return step
    img, ncls = (32, 10) if model_name == "vgg16" else (224, 1000)
    m = vgg16(nb_classes=ncls, input_shape=(img, img, 3)) if model_name == "vgg16" else ResNet50(
        input_shape=(img, img, 3), num_classes=ncls)
    m.compile(SGD(lr=0.01, momentum=0.9, weight_decay=5e-5), "sparse_categorical_crossentropy")
    m.place(dev, seed=0)
    ddp = DataParallel(m, comm.ProcessGroup(0, 1, 0, dev, None))
    stream = SyntheticImageStream(256, img, ncls, device=dev, seed=0, n_buffers=4)
    fn = CompiledTrainStep(m, warmup=2) if graph else ddp.train_step
    return lambda: fn(*stream.next())


def measure(step, K, KH=2):
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        step()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3 / K
    s_end = torch.cuda.Event(enable_timing=True)
    e_end = torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(int(2.0e9))  # ~1 s of GPU cycles: the host issues behind it
    s_end.record()
    t0 = time.perf_counter()
    for _ in range(KH):  # few steps: an eager step's launches must fit the HIP queue behind the sleep
        step()
    host = (time.perf_counter() - t0) * 1e3 / KH
    valid = not s_end.query()  # the sleep still running: the issue loop never waited on the device
    e_end.record()
    torch.cuda.synchronize()
    dev_ms = s_end.elapsed_time(e_end) / KH
    return {"wall_ms": round(wall, 3), "host_ms": round(host, 3), "host_valid": valid, "device_ms": round(dev_ms, 3)}


out = []
for name in sys.argv[1:] or ["vgg16", "resnet50"]:
    for graph in ((0,) if name == "bert" else (0, 1)):
        r = {"model": name, "graph": graph, **measure(build(name, graph), 50 if name == "vgg16" else 20)}
        print(json.dumps(r), flush=True)
