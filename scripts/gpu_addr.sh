#!/bin/bash
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/addr; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_transformer.py tests/test_gpu_hypothesis.py tests/test_gpu_gemm256.py tests/test_gpu_gemm_stream.py tests/test_gpu_layers.py > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python scripts/bench_wgrad.py > $O/wg.log 2>&1 || exit 1
grep shape $O/wg.log | cut -c1-90
for r in 1 2; do
  timeout -k 10 300 python bench.py --model bert --steps 10 --warmup 3 > $O/bert_$r.log 2>&1 || exit 1
  echo "bert $(tail -1 $O/bert_$r.log | grep -o '"value": [0-9.]*')"
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/rn_$r.log 2>&1 || exit 1
  echo "rn $(tail -1 $O/rn_$r.log | grep -o '"value": [0-9.]*')"
done
