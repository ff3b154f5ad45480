"""Yardstick probe: time torch.mm (hipBLASLt) on the BERT GEMM shapes so a kernel trace can name the library
kernel's tile configuration (macro tile, workgroup, LDS, VGPRs).  Not used by the framework."""
import torch

SHAPES = [(16384, 2304, 768), (16384, 3072, 768), (16384, 768, 3072), (16384, 768, 768), (8192, 8192, 8192)]


def main():
    for M, N, K in SHAPES:
        a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
        for _ in range(3):
            torch.mm(a, b.t())
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            torch.mm(a, b.t())
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 10
        print(f"{M}x{N}x{K} {ms:.4f} ms {2 * M * N * K / ms / 1e9:.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
