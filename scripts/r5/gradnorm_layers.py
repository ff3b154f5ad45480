"""Per-parameter gradient-norm ratio HIP (bf16) / CPU (fp32) of the small ResNet-50 step of
tests/test_gpu_kernels.py::test_resnet50_step_matches_reference: where does the HIP path lose norm?"""
import os
import sys

sys.path.insert(0, os.getcwd())
import torch

from distributeddeeplearningspark_amd.models import ResNet50

torch.manual_seed(0)
x = torch.randn(16, 64, 64, 3)
y = torch.randint(0, 10, (16,))
res = {}
for dev in ("cpu", "cuda"):
    m = ResNet50(input_shape=(64, 64, 3), num_classes=10)
    m.compile("sgd", "sparse_categorical_crossentropy")
    m.place(dev, seed=3)
    loss = m.backward_step(m.to_input(x), m.to_target(y))
    g = m.arena.to_canonical(m.arena.grad.detach()).float().cpu()
    res[dev] = (float(loss), g, m)
lc, gc, mc = res["cpu"]
lg, gg, _ = res["cuda"]
print(f"loss cpu {lc:.4f} gpu {lg:.4f}; grad norm cpu {gc.norm():.2f} gpu {gg.norm():.2f}")
rows = []
for p, co in zip(mc.arena.params, mc.arena.canon_offsets):
    a, b = gc[co:co + p.numel], gg[co:co + p.numel]
    na, nb = a.norm().item(), b.norm().item()
    cos = torch.nn.functional.cosine_similarity(a, b, dim=0).item() if na > 0 and nb > 0 else float("nan")
    rows.append((p.name, p.numel, na, nb, nb / na if na else float("nan"), cos))
tot_c = sum(r[2] ** 2 for r in rows)
print(f"{'param':44s} {'numel':>8s} {'|g| cpu':>10s} {'|g| gpu':>10s} {'ratio':>7s} {'cos':>7s} {'share':>6s}")
for r in rows:
    print(f"{r[0][:44]:44s} {r[1]:8d} {r[2]:10.4f} {r[3]:10.4f} {r[4]:7.4f} {r[5]:7.4f} {r[2] ** 2 / tot_c:6.3f}")
# aggregate by kind
import collections
agg = collections.defaultdict(lambda: [0.0, 0.0])
for r in rows:
    k = r[0].split("/")[-1]
    agg[k][0] += r[2] ** 2
    agg[k][1] += r[3] ** 2
for k, (a, b) in agg.items():
    print(f"kind {k:20s} norm cpu {a ** 0.5:10.3f} gpu {b ** 0.5:10.3f} ratio {(b / a) ** 0.5:.4f}")
