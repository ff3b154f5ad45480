"""3x3 convolution kernels of ResNet-50 (batch 256): forward, data-gradient and weight-gradient
of one conv per stage, 5 reps each — the workload for PMC counter runs (scripts/pmc_conv.sh)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributeddeeplearningspark_amd.ops import conv as CV

SHAPES = [(56, 64), (28, 128), (14, 256), (7, 512)]


def main():
    N = int(os.environ.get("BATCH", "256"))
    for H, C in SHAPES:
        g = CV.geometry(N, H, H, C, C, 3, 3, (1, 1), (1, 1), (1, 1))
        x = torch.randn(N, H, H, C, device="cuda").to(torch.bfloat16)
        w = (torch.randn(C, 3, 3, C, device="cuda") * 0.05).to(torch.bfloat16)
        dy = torch.randn(N, H, H, C, device="cuda").to(torch.bfloat16)
        gw = torch.zeros(C, 3, 3, C, device="cuda")
        for _ in range(5):
            CV.conv_fwd_native(x, w, g)
            CV.conv_dgrad_native(dy, w, g)
            CV.conv_wgrad_native(dy, x, g, gw)
        torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
