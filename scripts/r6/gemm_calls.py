"""Log every ops.gemm.gemm call of one eager ResNet-50 (or BERT) training step with its tile, split and grid
size in workgroup rounds (3 or 4 resident per CU), to find quantised grids.  Usage: gemm_calls.py [resnet50|bert]"""
import collections
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from distributeddeeplearningspark_amd.ops import gemm as G

calls = []
_orig = G.gemm


def spy(a, b, c, M, N, K, a_mode, b_mode, lda, ldb, ldc, epi, **kw):
    calls.append((M, N, K, a_mode, b_mode, epi, kw.get("tile"), kw.get("k_split"), kw.get("geom") is not None,
                  kw.get("stats") is not None, kw.get("bnr") is not None))
    return _orig(a, b, c, M, N, K, a_mode, b_mode, lda, ldb, ldc, epi, **kw)


G.gemm = spy


def main():
    model_name = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    dev = torch.device("cuda:0")
    from distributeddeeplearningspark_amd.parallel import comm
    from distributeddeeplearningspark_amd.parallel.ddp import DataParallel
    if model_name == "bert":
        from distributeddeeplearningspark_amd.data.synthetic import mlm_batch
        from distributeddeeplearningspark_amd.models.bert import BertConfig, BertForMaskedLM
        from distributeddeeplearningspark_amd.models.optimizers import AdamW
        cfg = BertConfig()
        m = BertForMaskedLM(cfg)
        m.compile(AdamW(lr=1e-4, weight_decay=0.01), "sparse_categorical_crossentropy")
        m.place(dev, seed=0)
        x, y = mlm_batch(32, 512, cfg.vocab_size, seed=0)
        x, y = m.to_input(x), m.to_target(y)
    else:
        from distributeddeeplearningspark_amd.data.ingest import SyntheticImageStream
        from distributeddeeplearningspark_amd.models import ResNet50
        from distributeddeeplearningspark_amd.models.optimizers import SGD
        m = ResNet50(input_shape=(224, 224, 3), num_classes=1000)
        m.compile(SGD(lr=0.1, momentum=0.9, weight_decay=5e-5), "sparse_categorical_crossentropy")
        m.place(dev, seed=0)
        x, y = SyntheticImageStream(256, 224, 1000, device=dev, seed=0, n_buffers=2).next()
    ddp = DataParallel(m, comm.ProcessGroup(0, 1, 0, dev, None))
    ddp.train_step(x, y)
    torch.cuda.synchronize()
    calls.clear()
    ddp.train_step(x, y)
    torch.cuda.synchronize()
    agg = collections.Counter(calls)
    for (M, N, K, am, bm, epi, tile, ks, geom, st, bnr), n in sorted(agg.items(), key=lambda kv: -kv[0][0] * kv[0][1] * kv[0][2]):
        print(f"{n:3d}x M={M:7d} N={N:5d} K={K:7d} A={am} B={bm} epi={epi} tile={tile} ks={ks} geom={int(geom)} "
              f"stats={int(st)} bnr={int(bnr)} gflop={2 * M * N * K / 1e9:7.1f}")


if __name__ == "__main__":
    main()
