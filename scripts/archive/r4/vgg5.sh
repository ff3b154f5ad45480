#!/bin/bash
# VGG-16 CIFAR batch 256: five runs on one box (median / spread), eager and hipGraph replay.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r4/vgg5; mkdir -p $O
for g in 0 1; do
  for i in 1 2 3 4 5; do
    timeout -k 10 200 python bench.py --model vgg16 --graph $g --steps 30 --warmup 5 2>/dev/null > $O/b.json || exit 1
    echo "graph=$g $(cut -c1-130 $O/b.json)" | tee -a $O/bench.txt
  done
done
