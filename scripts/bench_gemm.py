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
    # weight gradients: dW[N_out, K_in] += dY^T X over the token / pixel dimension (RC x RC, fp32, split-K)
    ("bert_qkv_wgrad", 2304, 768, T, G.RC, G.RC, "f32"),
    ("bert_ffn1_wgrad", 3072, 768, T, G.RC, G.RC, "f32"),
    ("bert_ffn2_wgrad", 768, 3072, T, G.RC, G.RC, "f32"),
    ("rn50_wgrad_1x1_64to256", 256, 64, 802816, G.RC, G.RC, "f32"),
    ("rn50_wgrad_1x1_1024to256", 256, 1024, 50176, G.RC, G.RC, "f32"),
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
    for shp in _shapes(sys.argv[1:]):
        name, M, N, K, am, bm = shp[:6]
        f32 = len(shp) > 6 and shp[6] == "f32"
        epi = G.EPI_F32 if f32 else G.EPI_BF16
        A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        B = torch.randn(N, K, device="cuda").to(torch.bfloat16)
        a_t = A if am == G.KC else A.T.contiguous()
        b_t = B if bm == G.KC else B.T.contiguous()
        out = torch.zeros(M, N, dtype=torch.float32 if f32 else torch.bfloat16, device="cuda")
        ref = (A[:256].float() @ B.float().T)
        runs = {}
        variants = {"g256": G.TILE256, "t128": G.choose_tile(M, N)}
        if f32:  # weight gradients: the production tile choice (gemm picks tile and split-K) and 128x128
            variants = {"auto": None, "t128": 0}
        elif not (M >= 256 and N >= 256 and K % 64 == 0):
            variants.pop("g256")
        def run(tile):
            if f32 and tile is None:  # the production call (tile, split-K rounds, slabs / atomics)
                return G.linear_wgrad(a_t, b_t, out)
            return G.gemm(a_t, b_t, out, M, N, K, am, bm, a_t.stride(0), b_t.stride(0), N, epi,
                          beta=1.0 if f32 else 0.0, tile=tile)
        for v, tile in variants.items():
            out.zero_()
            run(tile)
            err = ((out[:256].float() - ref).norm() / ref.norm()).item()
            runs[v] = {"err": err, "ms": []}
        runs["torch"] = {"ms": []}
        for _ in range(5):
            for v, tile in variants.items():
                runs[v]["ms"].append(timeit(lambda: run(tile)))
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
