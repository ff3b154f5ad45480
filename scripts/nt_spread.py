"""Run-to-run spread of the small ResNet-50 step (64x64, batch 16) on the HIP path with the BN sweeps'
plain vs nontemporal stores (DDL_BN_NT is read per launch): loss and gradient norm per run, to tell the
store form apart from the BN-statistics-atomics spread (test_resnet50_step_matches_reference)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributeddeeplearningspark_amd.models import ResNet50


def main():
    torch.manual_seed(0)
    x = torch.randn(16, 64, 64, 3)
    y = torch.randint(0, 10, (16,))
    m = ResNet50(input_shape=(64, 64, 3), num_classes=10)
    m.compile("sgd", "sparse_categorical_crossentropy")
    m.place("cuda:0", seed=3)
    xi, yt = m.to_input(x), m.to_target(y)
    out = {}
    for rep in range(4):
        for nt in ("0", "1"):
            os.environ["DDL_BN_NT"] = nt
            loss = m.backward_step(xi, yt)
            g = m.arena.grad.clone()
            out.setdefault(nt, []).append((round(float(loss), 5), round(g.norm().item(), 3)))
            out.setdefault(nt + "_grads", []).append(g)
    g0, g1 = out.pop("0_grads"), out.pop("1_grads")
    out["max_rel_diff_nt0_runs"] = max(((a - g0[0]).norm() / g0[0].norm()).item() for a in g0[1:])
    out["max_rel_diff_nt1_vs_nt0"] = max(((a - g0[0]).norm() / g0[0].norm()).item() for a in g1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
