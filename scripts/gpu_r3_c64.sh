#!/bin/bash
# 64-channel 3x3 resident-filter kernel: tests, microbenchmark vs the implicit GEMM, interleaved ResNet-50 A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "c64 or halo_kernel or dgrad_fused or bottleneck or resnet50_step or per_layer" > gpurun_out/c64_tests.log 2>&1
rc=$?; tail -3 gpurun_out/c64_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error" gpurun_out/c64_tests.log | head -20; exit $rc; }
: > gpurun_out/c64_micro.jsonl
for v in 1 0; do
  DDL_CONV3X3_C64PP=$v timeout -k 10 200 python scripts/bench_c64.py >> gpurun_out/c64_micro.jsonl 2>&1 || { tail gpurun_out/c64_micro.jsonl; exit 1; }
done
grep '^{' gpurun_out/c64_micro.jsonl
OUT=gpurun_out/ab_c64.jsonl; : > $OUT
for r in 1 2; do
  for cfg in "DDL_CONV3X3_C64PP=1" "DDL_CONV3X3_C64PP=0"; do
    env $cfg timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/ab_tmp.log 2>&1 || { echo "bench $cfg failed"; tail -20 gpurun_out/ab_tmp.log; exit 1; }
    line=$(grep '^{' gpurun_out/ab_tmp.log | tail -1)
    echo "{\"round\": $r, \"cfg\": \"$cfg\", \"bench\": $line}" >> $OUT
    echo "r$r $cfg $(echo $line | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
  done
done
for cfg in "DDL_CONV3X3_C64PP=1" "DDL_CONV3X3_C64PP=0"; do
  env $cfg timeout -k 10 300 python bench.py --model vgg16 --steps 30 --warmup 5 > gpurun_out/ab_tmp.log 2>&1 || { echo "vgg $cfg failed"; tail -20 gpurun_out/ab_tmp.log; exit 1; }
  echo "vgg $cfg $(grep '^{' gpurun_out/ab_tmp.log | tail -1 | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
done
