#!/bin/bash
# Persistent 256x256 ping-pong GEMM (tile 9): correctness, then the GEMM micro-benchmark on the BERT shapes.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4/persist
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm256.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4/persist/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4/persist/tests.log
[ $rc -ne 0 ] && exit $rc
DDL_BENCH_W4=0 timeout -k 10 300 python scripts/bench_gemm.py square_8192,square_4096,bert_qkv_fwd,bert_ffn1_fwd,bert_ffn2_fwd,bert_ffn1_dgrad,bert_ffn2_dgrad,rn50_l3_1x1_256to1024 > gpurun_out/r4/persist/gemm.jsonl 2>&1 || exit 1
python -c "
import json
for l in open('gpurun_out/r4/persist/gemm.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], {k:d[k]['tflops'] for k in d if isinstance(d[k], dict)})"
