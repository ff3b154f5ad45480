"""BERT-base Linear weight-gradient GEMMs (dW[N,K] += dY[M,N]^T X[M,K], fp32 accumulation):
hand-written split-K MFMA kernel vs hipBLASLt (torch.mm with an fp32 output).  Prints JSON lines."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributeddeeplearningspark_amd.ops import gemm as G

T = 16384
SHAPES = [("qkv", 2304, 768), ("out", 768, 768), ("ffn1", 3072, 768), ("ffn2", 768, 3072)]


def timeit(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    torch.manual_seed(0)
    for name, N, K in SHAPES:
        dy = torch.randn(T, N, device="cuda").to(torch.bfloat16)
        x = torch.randn(T, K, device="cuda").to(torch.bfloat16)
        gw = torch.zeros(N, K, device="cuda")
        ref = dy.float().t() @ x.float()
        G.linear_wgrad(dy, x, gw)
        err_ours = float((gw - ref).norm() / ref.norm())
        gw2 = torch.mm(dy.t(), x, out_dtype=torch.float32)
        err_blas = float((gw2 - ref).norm() / ref.norm())
        fl = 2.0 * T * N * K
        t_ours = timeit(lambda: G.linear_wgrad(dy, x, gw))
        t_blas = timeit(lambda: gw.add_(torch.mm(dy.t(), x, out_dtype=torch.float32)))
        t_blas_only = timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
        print(json.dumps({"shape": name, "N": N, "K": K, "M": T,
                          "ours_ms": round(t_ours, 4), "ours_tflops": round(fl / t_ours / 1e9, 1), "err_ours": err_ours,
                          "blas_add_ms": round(t_blas, 4), "blas_ms": round(t_blas_only, 4),
                          "blas_tflops": round(fl / t_blas_only / 1e9, 1), "err_blas": err_blas}), flush=True)


if __name__ == "__main__":
    main()
