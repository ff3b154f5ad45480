#!/bin/bash
# Row epilogue (EPI_BF16_ROW, DDL_GEMM_ROW_EPI=1) vs the unrolled full epilogue: correctness with the row
# epilogue forced, then interleaved BERT / ResNet benches, then the plain-GEMM LITE vs FULL code-size A/B.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4/epi
export TMPDIR=/tmp
DDL_GEMM_ROW_EPI=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_transformer.py tests/test_gpu_gemm256.py -x -q --timeout 200 --timeout-method thread -k "linear or gemm or conv or transformer or bert or epilogue or attention or layer" > gpurun_out/r4/epi/tests_row.log 2>&1
rc=$?; tail -3 gpurun_out/r4/epi/tests_row.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for i in 1 2; do
  for v in 0 1; do
    DDL_GEMM_ROW_EPI=$v timeout -k 10 300 python bench.py --model bert --steps 10 --warmup 3 2>/dev/null | grep '^{' | sed "s/^/row=$v /" >> gpurun_out/r4/epi/bert_ab.txt || exit 1
    DDL_GEMM_ROW_EPI=$v timeout -k 10 300 python bench.py --steps 15 --warmup 4 2>/dev/null | grep '^{' | sed "s/^/row=$v /" >> gpurun_out/r4/epi/resnet_ab.txt || exit 1
  done
done
python - <<'PY'
import json
for f in ("bert_ab", "resnet_ab"):
    for line in open(f"gpurun_out/r4/epi/{f}.txt"):
        tag, js = line.split(" ", 1)
        d = json.loads(js)
        print(f, tag, round(d["value"]), d["ms_per_step"])
PY
timeout -k 10 300 python scripts/bench_gemm.py bert_qkv_fwd,bert_ffn1_fwd,bert_ffn2_fwd,bert_ffn1_dgrad,square_8192 > gpurun_out/r4/epi/gemm_lite.jsonl 2>&1 || exit 1
DDL_GEMM_FULL_EPI=1 timeout -k 10 300 python scripts/bench_gemm.py bert_qkv_fwd,bert_ffn1_fwd,bert_ffn2_fwd,bert_ffn1_dgrad,square_8192 > gpurun_out/r4/epi/gemm_full.jsonl 2>&1 || exit 1
DDL_GEMM_FULL_EPI=1 DDL_GEMM_ROW_EPI=1 timeout -k 10 300 python scripts/bench_gemm.py bert_qkv_fwd,bert_ffn1_fwd,bert_ffn2_fwd,bert_ffn1_dgrad,square_8192 > gpurun_out/r4/epi/gemm_row.jsonl 2>&1 || exit 1
for f in lite full row; do echo "== $f"; python -c "
import json,sys
for l in open('gpurun_out/r4/epi/gemm_$f.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], {k:d[k]['tflops'] for k in ('g256','t128','torch') if k in d})"; done
# split-K slabs vs fp32 atomics (weight gradients): test, then interleaved BERT / ResNet A/B
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "slabs" > gpurun_out/r4/epi/tests_slabs.log 2>&1
src=$?; tail -2 gpurun_out/r4/epi/tests_slabs.log
[ $src -ne 0 ] && [ $src -ne 1 ] && exit $src
for i in 1 2; do
  for v in 0 1; do
    DDL_SPLITK_SLABS=$v timeout -k 10 300 python bench.py --model bert --steps 10 --warmup 3 2>/dev/null | grep '^{' | sed "s/^/slabs=$v /" >> gpurun_out/r4/epi/bert_slabs.txt || exit 1
    DDL_SPLITK_SLABS=$v timeout -k 10 300 python bench.py --steps 15 --warmup 4 2>/dev/null | grep '^{' | sed "s/^/slabs=$v /" >> gpurun_out/r4/epi/resnet_slabs.txt || exit 1
  done
done
python - <<'PY'
import json
for f in ("bert_slabs", "resnet_slabs"):
    for line in open(f"gpurun_out/r4/epi/{f}.txt"):
        tag, js = line.split(" ", 1)
        d = json.loads(js)
        print(f, tag, round(d["value"]), d["ms_per_step"])
PY
exit $rc
