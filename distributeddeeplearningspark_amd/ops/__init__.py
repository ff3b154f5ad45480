"""Op layer: every op dispatches to the HIP kernels on GPU tensors and to a PyTorch
reference on CPU tensors (the reference doubles as the numerics oracle in tests)."""
from ._native import has_native, use_native  # noqa: F401
