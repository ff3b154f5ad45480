#!/bin/bash
# hipGraph replay of the whole 1-GPU step vs eager launches, interleaved after a warm-up run.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/graph2; mkdir -p $O
timeout -k 10 300 python bench.py --model vgg16 --steps 10 --warmup 3 > $O/warm.log 2>&1 || { tail $O/warm.log; exit 1; }
for r in 1 2; do
  for g in 0 1; do
    for m in vgg16 resnet50; do
      timeout -k 10 300 python bench.py --model $m --graph $g --steps 30 --warmup 5 > $O/${m}_g${g}_$r.log 2>&1 || { tail $O/${m}_g${g}_$r.log; exit 1; }
      echo "$m graph=$g r=$r $(tail -1 $O/${m}_g${g}_$r.log | grep -o '"value": [0-9.]*')"
    done
  done
done
