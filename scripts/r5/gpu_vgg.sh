#!/bin/bash
# VGG-16: conv-chain BN-reduce fusion tests, five bench runs, steady-state launches; BERT bench x2.
export TMPDIR=/tmp
O=gpurun_out/r5/vgg
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_layers.py tests/test_gpu_stem.py tests/test_gpu_kernels.py \
  -k "sequential or chain or s2d or zero_ranges or stem or pool or vgg" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2 3 4 5; do
  timeout -k 10 200 python bench.py --model vgg16 > $O/vgg16_bench_$i.log 2>&1 || exit 1
  tail -1 $O/vgg16_bench_$i.log | cut -c1-110
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --model bert --steps 10 --warmup 3 > $O/bert_bench_$i.log 2>&1 || exit 1
  tail -1 $O/bert_bench_$i.log | cut -c1-110
done
MODELS="vgg16" bash scripts/r5/launch_count.sh || exit 1
