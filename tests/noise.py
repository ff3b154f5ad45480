"""Model-level A/B comparisons against the run-to-run noise floor.

A bf16 ResNet training step is not bitwise reproducible: the BN statistics are accumulated with
fp32 atomics (order-dependent at ~1e-7 relative), and every bf16 rounding downstream turns such a
perturbation delta into sparse one-ulp flips of norm ~sqrt(delta * ulp).  Measured on MI355X for a
ResNet(blocks=(2, 2)) forward at 64x64 (scripts/diag_determinism.py): the same input through the same
kernels differs by 7e-6, 3e-4, 2.7e-3, 5.6e-3 (relative norm) after blocks 1..4, while every conv's
pre-BN output is bitwise identical.  A fixed tolerance on a two-variant comparison is therefore
either loose or flaky; these helpers compare the variant under test with the reference variant's own
spread (two reference runs) instead."""
from __future__ import annotations


def rel(a, b) -> float:
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def assert_within_noise(test, ref_a, ref_b, floor: float, factor: float = 4.0, what: str = ""):
    """``test`` (tensor) vs ``ref_a``: relative-norm distance <= factor x max(spread(ref_a, ref_b), floor)."""
    spread = rel(ref_b, ref_a)
    d = rel(test, ref_a)
    assert d <= factor * max(spread, floor), f"{what}: rel diff {d:.3e} vs reference spread {spread:.3e} (floor {floor})"
    return d, spread


def assert_scalar_within_noise(test: float, ref_a: float, ref_b: float, floor: float, factor: float = 4.0,
                               what: str = "loss"):
    spread = abs(ref_b - ref_a)
    d = abs(test - ref_a)
    lim = factor * max(spread, floor * max(1.0, abs(ref_a)))
    assert d <= lim, f"{what}: |diff| {d:.3e} vs reference spread {spread:.3e} (limit {lim:.3e})"
    return d, spread
