#!/bin/bash
# GEMM knob sweep on the BERT / ResNet shapes (forward, data- and weight-gradients): default vs the
# double-stage LDS-DMA kernel, split-K slabs, and the 128x128 weight-gradient tile.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4/gemm
S=bert_qkv_fwd,bert_ffn1_fwd,bert_ffn2_fwd,bert_ffn1_dgrad,bert_ffn2_dgrad,bert_qkv_wgrad,bert_ffn1_wgrad,bert_ffn2_wgrad,rn50_wgrad_1x1_64to256,rn50_wgrad_1x1_1024to256,rn50_l3_1x1_1024to256
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python scripts/bench_gemm.py $S > gpurun_out/r4/gemm/$tag.jsonl 2>&1 || return 1
  python -c "
import json
for l in open('gpurun_out/r4/gemm/$tag.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('$tag', d['shape'], {k:d[k]['tflops'] for k in d if isinstance(d[k], dict)})"; }
run default DDL_X=0 && run ring3 DDL_GEMM_STAGES=3 && run ring4 DDL_GEMM_STAGES=4 && run dma2 DDL_GEMM_DMA=2 && run wg_ring3 DDL_WGRAD_STAGES=3 && run slabs DDL_SPLITK_SLABS=1 && run slabs_r2 DDL_SPLITK_SLABS=1 DDL_LINEAR_WGRAD_ROUNDS=2
