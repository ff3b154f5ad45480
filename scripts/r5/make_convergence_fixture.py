"""fp32 CPU reference curve of tests/test_gpu_convergence.py::test_resnet50_deterministic_convergence_vs_fp32_curve:
ResNet-50 (64x64, 10 classes) trained 150 steps of SGD(0.01, momentum 0.9) on the synthetic template task at
batch 32, on the CPU in fp32.  Writes tests/fixtures/resnet50_synthetic_fp32_curve.json."""
import json
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import numpy as np
import torch

sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from test_gpu_convergence import _batch, _templates  # noqa: E402

from distributeddeeplearningspark_amd.models import ResNet50  # noqa: E402
from distributeddeeplearningspark_amd.models.optimizers import SGD  # noqa: E402

torch.set_num_threads(8)
tmpl = _templates()
torch.manual_seed(0)
m = ResNet50(input_shape=(64, 64, 3), num_classes=10)
m.compile(SGD(lr=0.01, momentum=0.9), "sparse_categorical_crossentropy")
m.place("cpu", seed=1)
g = torch.Generator().manual_seed(2)
losses, t0 = [], time.time()
for i in range(150):
    x, y = _batch(tmpl, 32, g)
    losses.append(float(m.train_on_batch(m.to_input(x), m.to_target(y))))
    if i % 25 == 0:
        print(i, losses[-1], round(time.time() - t0, 1), flush=True)
xt, yt = _batch(tmpl, 512, torch.Generator().manual_seed(99))
acc = float((m.predict(xt.numpy(), batch_size=128).argmax(1) == yt.numpy()).mean())
out = {"model": "ResNet50(64x64x3, 10 classes)", "optimizer": "SGD(lr=0.01, momentum=0.9)", "batch": 32, "steps": 150,
       "device": "cpu", "dtype": "fp32", "losses": losses, "heldout_accuracy": acc,
       "generator": "scripts/r5/make_convergence_fixture.py"}
json.dump(out, open("tests/fixtures/resnet50_synthetic_fp32_curve.json", "w"))
print("accuracy", acc, "windows", [round(float(np.mean(losses[a:a + 10])), 3) for a in (0, 30, 70, 140)])
