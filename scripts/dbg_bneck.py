import sys, os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import os, torch
from distributeddeeplearningspark_amd.models.resnet import ResNet
torch.manual_seed(1)
x = torch.randn(16, 32, 32, 3); y = torch.randint(0, 10, (16,))
res = {}
for fused in ("1", "0"):
    os.environ["DDL_FUSED_BLOCKS"] = fused
    m = ResNet(blocks=(2,), input_shape=(32, 32, 3), num_classes=10)
    m.compile("sgd", "sparse_categorical_crossentropy"); m.place("cuda", seed=5)
    loss = m.backward_step(m.to_input(x), m.to_target(y))
    res[fused] = (float(loss), {p.name: p.grad.detach().float().cpu().clone() for p in m.arena.params if p.trainable})
print("loss", res["1"][0], res["0"][0])
for k in res["0"][1]:
    a, b = res["1"][1][k], res["0"][1][k]
    print(f"{k:40s} rel {((a-b).norm()/(b.norm()+1e-12)).item():.4f} norm {b.norm().item():.4e}")
