#!/bin/bash
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/bsk; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_transformer.py > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2; do
  for v in 1 0; do
    DDL_DGRAD_SPLITK=$v timeout -k 10 300 python bench.py --model bert --steps 10 --warmup 3 > $O/bert_${v}_$r.log 2>&1 || exit 1
    echo "splitk=$v $(tail -1 $O/bert_${v}_$r.log | grep -o '"value": [0-9.]*')"
  done
done
