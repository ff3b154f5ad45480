#!/bin/bash
# BN apply / dx sweeps with nontemporal output stores (DDL_BN_NT=1) vs plain stores: model-level GPU
# tests with NT on, then interleaved ResNet-50 and VGG-16 A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
DDL_BN_NT=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_layers.py -k "batchnorm or bn_ or bottleneck or sequential" > gpurun_out/bnnt_tests.log 2>&1
rc=$?; tail -1 gpurun_out/bnnt_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/bnnt_tests.log | head -20; exit $rc; }
OUT=gpurun_out/ab_bnnt.jsonl; : > $OUT
for r in 1 2 3; do
  for v in 1 0; do
    DDL_BN_NT=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_tmp.log 2>&1 || { tail gpurun_out/ab_tmp.log; exit 1; }
    line=$(grep '^{' gpurun_out/ab_tmp.log | tail -1)
    echo "{\"round\": $r, \"model\": \"resnet50\", \"DDL_BN_NT\": \"$v\", \"bench\": $line}" >> $OUT
    echo "r$r resnet50 nt=$v $(echo $line | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
  done
done
for r in 1 2; do
  for v in 1 0; do
    DDL_BN_NT=$v timeout -k 10 300 python bench.py --model vgg16 --steps 50 --warmup 10 > gpurun_out/ab_tmp.log 2>&1 || { tail gpurun_out/ab_tmp.log; exit 1; }
    line=$(grep '^{' gpurun_out/ab_tmp.log | tail -1)
    echo "{\"round\": $r, \"model\": \"vgg16\", \"DDL_BN_NT\": \"$v\", \"bench\": $line}" >> $OUT
    echo "r$r vgg16 nt=$v $(echo $line | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
  done
done
