#!/bin/bash
# XCD-aware attention block remap (DDL_ATTN_XCD) and GEMM raster group size: tests, microbench, BERT A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_transformer.py > gpurun_out/attn_tests.log 2>&1
rc=$?; tail -1 gpurun_out/attn_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/attn_tests.log | head; exit $rc; }
for v in 1 0; do
  DDL_ATTN_XCD=$v timeout -k 10 200 python scripts/bench_attention.py > gpurun_out/attn_micro_$v.txt 2>&1 || { tail gpurun_out/attn_micro_$v.txt; exit 1; }
  echo "XCD=$v"; grep -v amdgpu.ids gpurun_out/attn_micro_$v.txt | tail -4
done
OUT=gpurun_out/ab_attn_xcd.jsonl; : > $OUT
for r in 1 2; do
  for cfg in "DDL_ATTN_XCD=1" "DDL_ATTN_XCD=0" "DDL_ATTN_XCD=1 DDL_GEMM_GROUP_M=16"; do
    env $cfg timeout -k 10 300 python bench.py --model bert --steps 20 --warmup 3 > gpurun_out/ab_tmp.log 2>&1 || { tail gpurun_out/ab_tmp.log; exit 1; }
    line=$(grep '^{' gpurun_out/ab_tmp.log | tail -1)
    echo "{\"round\": $r, \"cfg\": \"$cfg\", \"bench\": $line}" >> $OUT
    echo "r$r $cfg $(echo $line | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
  done
done
