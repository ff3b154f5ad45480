"""Calibrate the well-conditioned per-stage gradient check (tests/test_gpu_determinism.py): per-stage
cosines of the fp32 CPU gradient against its 2^-7 / 2^-8 input-perturbed self and against the
deterministic HIP gradient, for several gamma3 values, plus the shortcut-mutation arm."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from test_gpu_determinism import DEV, _resnet50_conditioned, _stage_cosines  # noqa: E402

for g3 in (0.1, 0.05):
    m, lc, gc = _resnet50_conditioned("cpu", gamma3=g3)
    for nz in (2.0 ** -7, 2.0 ** -8):
        _, _, gp = _resnet50_conditioned("cpu", noise=nz, gamma3=g3)
        print(f"gamma3={g3} cpu vs perturbed {nz}:", {k: round(v, 4) for k, v in _stage_cosines(m, gc, gp).items()},
              flush=True)
    _, lg, gg = _resnet50_conditioned(DEV, gamma3=g3)
    print(f"gamma3={g3} gpu vs cpu:", {k: round(v, 4) for k, v in _stage_cosines(m, gc, gg).items()}, lc, lg, flush=True)
    _, _, gb = _resnet50_conditioned(DEV, gamma3=g3, mutation=("drop_shortcut", "resnet50/s3b6"))
    print(f"gamma3={g3} mutated gpu vs cpu:", {k: round(v, 4) for k, v in _stage_cosines(m, gc, gb).items()},
          flush=True)
