"""Time the stem's space-to-depth pad kernel (batch 256, 224x224x3 -> 115x115x16) with HIP events."""
import os
import sys

sys.path.insert(0, os.getcwd())
import torch

from distributeddeeplearningspark_amd.ops._native import C

x = torch.randn(256, 224, 224, 3, device="cuda").to(torch.bfloat16)
y = torch.empty(256, 115, 115, 16, dtype=torch.bfloat16, device="cuda")
for _ in range(5):
    C().s2d_pad(x, y, 3)
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(50):
    C().s2d_pad(x, y, 3)
b.record()
b.synchronize()
print(f"{os.getcwd()}: s2d_pad {a.elapsed_time(b) / 50 * 1e3:.1f} us")
