"""GEMM microbenchmark on random bf16 data: the 256x256 ping-pong kernel vs the 128-tile
kernel (and hipBLASLt via torch.matmul as an external yardstick) on BERT-base and
ResNet-50 shapes.  Interleaved rounds in one process; prints TFLOP/s medians as JSON lines."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributeddeeplearningspark_amd.ops import gemm as G

T = 16384
SHAPES = [  # name, M, N, K, a_mode, b_mode
    ("square_8192", 8192, 8192, 8192, G.KC, G.KC),
    ("square_4096", 4096, 4096, 4096, G.KC, G.KC),
    ("bert_qkv_fwd", T, 2304, 768, G.KC, G.KC),
    ("bert_ffn1_fwd", T, 3072, 768, G.KC, G.KC),
    ("bert_ffn2_fwd", T, 768, 3072, G.KC, G.KC),
    ("bert_ffn1_dgrad", T, 768, 3072, G.KC, G.RC),
    ("bert_ffn2_dgrad", T, 3072, 768, G.KC, G.RC),
    ("rn50_l1_1x1_64to256", 802816, 256, 64, G.KC, G.KC),
    ("rn50_l3_1x1_1024to256", 50176, 256, 1024, G.KC, G.KC),
    ("rn50_l3_1x1_256to1024", 50176, 1024, 256, G.KC, G.KC),
    ("rn50_l2_dgrad_512to128", 200704, 128, 512, G.KC, G.RC),
]


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


def _shapes(argv):
    """Named shapes (comma list) or ad-hoc ``MxNxK[:rc]`` entries (``:rc`` = B row-contiguous)."""
    if not argv:
        return SHAPES
    out = []
    for tok in argv[0].split(","):
        named = [s for s in SHAPES if s[0] == tok]
        if named:
            out += named
            continue
        dims, _, mode = tok.partition(":")
        M, N, K = (int(v) for v in dims.split("x"))
        out.append((tok, M, N, K, G.KC, G.RC if mode == "rc" else G.KC))
    return out


def main():
    torch.manual_seed(0)
    for name, M, N, K, am, bm in _shapes(sys.argv[1:]):
        A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        B = torch.randn(N, K, device="cuda").to(torch.bfloat16)
        a_t = A if am == G.KC else A.T.contiguous()
        b_t = B if bm == G.KC else B.T.contiguous()
        out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        ref = (A[:256].float() @ B.float().T)
        runs = {}
        variants = {"g256": G.TILE256, "t128": G.choose_tile(M, N)}
        if M >= 256 and N >= 256 and K % 64 == 0:
            pass
        else:
            variants.pop("g256")
        for v, tile in variants.items():
            G.gemm(a_t, b_t, out, M, N, K, am, bm, a_t.stride(0), b_t.stride(0), N, G.EPI_BF16, tile=tile)
            err = ((out[:256].float() - ref).norm() / ref.norm()).item()
            runs[v] = {"err": err, "ms": []}
        runs["torch"] = {"ms": []}
        for _ in range(5):
            for v, tile in variants.items():
                runs[v]["ms"].append(timeit(lambda: G.gemm(a_t, b_t, out, M, N, K, am, bm, a_t.stride(0),
                                                             b_t.stride(0), N, G.EPI_BF16, tile=tile)))
            runs["torch"]["ms"].append(timeit(lambda: torch.matmul(A, B.T)))
        flop = 2.0 * M * N * K
        res = {"shape": name, "M": M, "N": N, "K": K}
        for v, r in runs.items():
            ms = statistics.median(r["ms"])
            res[v] = {"ms": round(ms, 4), "tflops": round(flop / ms / 1e9, 1)}
            if "err" in r:
                res[v]["rel_err"] = round(r["err"], 5)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
