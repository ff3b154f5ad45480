"""BERT-MLM model and transformer reference ops on CPU (the GPU kernels are checked
against these in tests/test_gpu_transformer.py)."""
import math

import numpy as np
import torch

from distributeddeeplearningspark_amd.models.bert import BertConfig, BertForMaskedLM
from distributeddeeplearningspark_amd.ops import transformer as T


def test_dropout_hash_mask_statistics_and_determinism():
    idx = torch.arange(200_000)
    k1 = T.keep_mask_ref(42, idx, 0.1)
    k2 = T.keep_mask_ref(42, idx, 0.1)
    k3 = T.keep_mask_ref(43, idx, 0.1)
    assert torch.equal(k1, k2)
    assert abs(k1.float().mean().item() - 0.9) < 0.005
    assert (k1 != k3).float().mean().item() > 0.1  # different seed, different mask
    # the dropout bytes behave uniformly
    u = T.drop_hash_ref(7, idx).double() / 256
    assert abs(u.mean().item() - 255 / 512) < 0.01
    assert T.drop_thresh(0.1) == 26 and T.drop_thresh(0.25) == 64 and T.drop_scale(0.25) == 256 / 192


def _drop_byte_py(seed: int, idx: int) -> int:
    """Plain-integer transcription of ddl_common.h drop_keep's byte (uint64 / uint32 wraparound)."""
    M32 = 0xFFFFFFFF
    q = (seed + (idx >> 2)) & 0xFFFFFFFFFFFFFFFF
    x = ((q & M32) ^ (((q >> 32) & 0xFFFFFF) * 0x9E3779 & M32)) * 0x9E3779B1 & M32
    x ^= x >> 16
    x = (x & 0xFFFFFF) * 0x7FEB35 & M32
    x ^= x >> 15
    x = (x & 0xFFFFFF) * 0x846CA7 & M32
    x ^= x >> 16
    return (x >> (8 * (idx & 3))) & 0xFF


def test_dropout_hash_ref_matches_integer_transcription():
    """The int64-tensor reference (signed wraparound) equals the unsigned integer definition, for seeds
    that overflow int64 and element indices past 2^32."""
    rng = np.random.default_rng(5)
    for seed in (0, 7, 2**40 + 3, 2**63 + 12345, 2**64 - 5):
        idx = [int(v) for v in rng.integers(0, 2**34, size=64)] + [0, 1, 2, 3, 4, 5]
        got = T.drop_hash_ref(seed, torch.tensor(idx, dtype=torch.int64)).tolist()
        assert got == [_drop_byte_py(seed, i) for i in idx], seed


def test_attention_ref_matches_sdpa():
    B, S, H = 2, 16, 3
    qkv = torch.randn(B * S, 3 * H * 64)
    o = T.attention_ref(qkv, B, S, H, 0, H * 64, 2 * H * 64)
    x = qkv.view(B, S, 3, H, 64).permute(2, 0, 3, 1, 4)
    ref = torch.nn.functional.scaled_dot_product_attention(x[0], x[1], x[2])
    np.testing.assert_allclose(o.numpy(), ref.permute(0, 2, 1, 3).reshape(B * S, -1).numpy(), atol=1e-5)


def test_attention_ref_key_padding():
    B, S, H = 2, 8, 1
    qkv = torch.randn(B * S, 3 * 64)
    lens = torch.tensor([8, 5], dtype=torch.int32)
    o = T.attention_ref(qkv, B, S, H, 0, 64, 128, lens)
    # changing padded keys/values of sequence 1 must not change its outputs
    q2 = qkv.clone()
    q2[S + 5:, 64:] = torch.randn(3, 128)
    o2 = T.attention_ref(q2, B, S, H, 0, 64, 128, lens)
    np.testing.assert_allclose(o[S:].numpy(), o2[S:].numpy(), atol=1e-6)


def _batch(cfg, B=4, S=128, P=20, seed=0):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(0, cfg.vocab_size, (B, S), generator=g)
    pos = torch.stack([torch.randperm(S, generator=g)[:P].sort().values for _ in range(B)])
    return {"input_ids": ids}, {"positions": pos, "labels": torch.gather(ids, 1, pos), "num_masked": B * P}


def test_bert_tiny_trains_on_cpu():
    cfg = BertConfig.tiny()
    m = BertForMaskedLM(cfg)
    m.compile("adamw", "sparse_categorical_crossentropy")
    m.place("cpu", seed=0)
    x, y = _batch(cfg)
    losses = [m.train_on_batch(x, y) for _ in range(6)]
    assert abs(losses[0] - math.log(cfg.vocab_size)) < 1.0
    assert losses[-1] < losses[0] - 0.5, losses


def test_bert_param_count_base():
    m = BertForMaskedLM(BertConfig())
    m.build_model()
    # HF bert-base-uncased MLM: 109,514,298 incl. the tied decoder once; our word table is
    # stored padded to 30528 rows (+6*768) and the decoder bias to 30528 (+6)
    assert m.count_params() == 109_514_298 + 6 * 768 + 6


def test_bert_full_logits_and_dropout_off_in_eval():
    cfg = BertConfig.tiny(num_hidden_layers=1)
    m = BertForMaskedLM(cfg)
    m.place("cpu", seed=1)
    x, _ = _batch(cfg, B=2, S=128)
    a = m.forward(x)
    b = m.forward(x)
    assert a.shape == (2, 128, cfg.vocab_size)
    assert torch.equal(a, b)
