"""Run the fused ResNet training forward twice on the same input and report, stage by stage, how far
the two runs' activations differ (atomics in the BN statistics give ~1e-6; a race gives far more)."""
import sys

import torch

sys.path.insert(0, ".")
from distributeddeeplearningspark_amd.models.resnet import ResNet  # noqa: E402
from distributeddeeplearningspark_amd.ops import pool as pool_ops  # noqa: E402
from distributeddeeplearningspark_amd.ops.fused_blocks import stem_pool  # noqa: E402
from distributeddeeplearningspark_amd.ops.norm import reset_workspaces  # noqa: E402

DEV = "cuda:0"
blocks = tuple(int(b) for b in (sys.argv[1] if len(sys.argv) > 1 else "2,2").split(","))
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
H = int(sys.argv[3]) if len(sys.argv) > 3 else 64
torch.manual_seed(4)
x = torch.randn(B, H, H, 3)
m = ResNet(blocks=blocks, input_shape=(H, H, 3), num_classes=10)
m.compile("sgd", "sparse_categorical_crossentropy")
m.place(DEV, seed=5)
xd = m.to_input(x)


def run():
    reset_workspaces(DEV)
    outs = []
    with torch.no_grad():
        y = stem_pool(m.stem, xd, m.stem.conv.kernel.data)
        outs.append(("stem_pool", y.float().clone()))
        for b in m.stages:
            y = b.call(y, True)
            outs.append((b.name, y.float().clone()))
    torch.cuda.synchronize()
    return outs


runs = [run() for _ in range(3)]
for i, (name, a) in enumerate(runs[0]):
    for r in (1, 2):
        b = runs[r][i][1]
        d = (a - b).abs()
        print(f"{name:24s} run0 vs run{r}: max {d.max().item():.3e} rel {(d.norm() / a.norm()).item():.3e} "
              f"nbad {(d > 1e-2 * a.abs().max()).sum().item()}", flush=True)

# per-unit: the same input through each conv twice -> pre-BN outputs must be bitwise equal
from distributeddeeplearningspark_amd.ops.fused_blocks import convbn_forward  # noqa: E402

print("--- per-unit conv determinism (same input) ---")
with torch.no_grad():
    y = stem_pool(m.stem, xd, m.stem.conv.kernel.data)
    for b in m.stages:
        for uname in ("down", "c1", "c2", "c3"):
            unit = getattr(b, uname)
            if unit is None:
                continue
            inp = y
            if uname == "c2":
                inp = convbn_forward(b.c1, y).y
            if uname == "c3":
                inp = convbn_forward(b.c2, convbn_forward(b.c1, y).y).y
            res = []
            for _ in range(3):
                reset_workspaces(DEV)
                st = convbn_forward(unit, inp.clone(), relu=uname != "down", apply=uname != "down")
                torch.cuda.synchronize()
                res.append((st.yc.float().clone(), st.scale.clone(), st.mean.clone()))
            for r in (1, 2):
                dyc = (res[0][0] - res[r][0]).abs().max().item()
                dsc = ((res[0][1] - res[r][1]).abs() / res[0][1].abs().clamp_min(1e-12)).max().item()
                print(f"{b.name}/{uname} {tuple(inp.shape)}->{tuple(res[0][0].shape)} yc maxdiff {dyc:.3e} "
                      f"scale reldiff {dsc:.3e}", flush=True)
        y = b.call(y, True)
