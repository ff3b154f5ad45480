"""fp32 CPU envelope for tests/test_gpu_convergence.py::test_resnet50_curve_inside_fp32_envelope.

ResNet-50 (64x64, 10 classes) trained STEPS steps of SGD(LR, momentum 0.9) at batch 32 on the hard synthetic
template task (tests/test_gpu_convergence.py::_hard_batch: noise NOISE, so the loss is still falling at step 100),
on the CPU in fp32, K times: run 0 from the unperturbed initial weights, runs 1..K-1 with every initial weight
multiplied by (1 + 1e-3 * N(0, 1)) (seeded) — the size of a bf16 rounding — so the spread of the K curves is
the natural sensitivity of this trajectory.  Writes tests/fixtures/resnet50_hard_fp32_envelope.json.
Usage: python scripts/r6/make_envelope_fixture.py [K] [STEPS]"""
import json
import os
import sys
import time

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np
import torch

from test_gpu_convergence import HARD, _hard_batch, _templates  # noqa: E402

from distributeddeeplearningspark_amd.models import ResNet50  # noqa: E402
from distributeddeeplearningspark_amd.models.optimizers import SGD  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 4
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else HARD["steps"]
torch.set_num_threads(8)
tmpl = _templates(classes=HARD["classes"])
curves = []
for k in range(K):
    torch.manual_seed(0)
    m = ResNet50(input_shape=(64, 64, 3), num_classes=HARD["classes"])
    m.compile(SGD(lr=HARD["lr"], momentum=0.9), "sparse_categorical_crossentropy")
    m.place("cpu", seed=1)
    if k:
        g = torch.Generator().manual_seed(1000 + k)
        with torch.no_grad():
            w = m.arena.master
            w.mul_(1 + 1e-3 * torch.randn(w.shape, generator=g))
            m.arena.sync_compute()
    g = torch.Generator().manual_seed(2)
    losses, t0 = [], time.time()
    for i in range(STEPS):
        x, y = _hard_batch(tmpl, 32, g)
        losses.append(float(m.train_on_batch(m.to_input(x), m.to_target(y))))
        if i % 25 == 0:
            print(k, i, round(losses[-1], 4), round(time.time() - t0, 1), flush=True)
    curves.append(losses)
    print("run", k, "windows", [round(float(np.mean(losses[a:a + 10])), 3) for a in range(0, STEPS, 10)], flush=True)
out = {"model": f"ResNet50(64x64x3, {HARD['classes']} classes)", "optimizer": f"SGD(lr={HARD['lr']}, momentum=0.9)",
       "batch": 32, "steps": STEPS, "noise": HARD["noise"], "device": "cpu", "dtype": "fp32",
       "perturbation": "initial weights x (1 + 1e-3 N(0,1)), runs 1..K-1", "curves": curves,
       "generator": "scripts/r6/make_envelope_fixture.py"}
if len(sys.argv) <= 3:
    json.dump(out, open("tests/fixtures/resnet50_hard_fp32_envelope.json", "w"))
