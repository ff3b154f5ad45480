#!/bin/bash
# hipGraph-replayed step (--graph 1) vs eager launches, ResNet-50 and VGG-16, one GPU
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/graph; mkdir -p $O
for m in resnet50 vgg16; do
  for g in 0 1; do
    timeout -k 10 300 python bench.py --model $m --graph $g --steps 20 --warmup 5 > $O/${m}_g$g.log 2>&1 || { tail -5 $O/${m}_g$g.log; exit 1; }
    echo "$m graph=$g $(tail -1 $O/${m}_g$g.log | cut -c60-130)"
  done
done
