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
            loss = m.backward_step(xi, yt).detach()
            g = m.arena.grad.clone()
            out.setdefault(nt, []).append((round(float(loss), 5), round(g.norm().item(), 3)))
            out.setdefault(nt + "_grads", []).append(g)
    g0, g1 = out.pop("0_grads"), out.pop("1_grads")
    rel = lambda a, b: round(((a - b).norm() / b.norm()).item(), 5)
    out["rel_diff_nt0_consecutive"] = [rel(g0[i + 1], g0[i]) for i in range(len(g0) - 1)]
    out["rel_diff_nt1_vs_nt0_same_rep"] = [rel(a, b) for a, b in zip(g1, g0)]
    # where along the arena the runs part (the arena's layer order: first decile = stem side)
    n = g0[0].numel()
    out["rel_diff_by_arena_decile_nt0"] = [rel(g0[1][k * n // 10:(k + 1) * n // 10], g0[0][k * n // 10:(k + 1) * n // 10])
                                           for k in range(10)]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
