#!/bin/bash
# Whole-step hipGraph replay (--graph 1) vs eager launches on ResNet-50 and VGG-16, interleaved on one box.
set -o pipefail
mkdir -p gpurun_out/r6
out=gpurun_out/r6/ab_graph.txt
: > $out
for r in 1 2; do
  for g in 0 1; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --graph $g 2>/dev/null | sed "s/^/rn50 graph=$g /" >> $out || exit 1
    timeout -k 10 200 python -u bench.py --model vgg16 --steps 50 --warmup 10 --graph $g 2>/dev/null | sed "s/^/vgg16 graph=$g /" >> $out || exit 1
  done
done
