#!/bin/bash
# Interleaved A/B against a previous build in ab_prev/ (see the commit message of the run), BERT-base and ResNet-50.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r4/ab_prev; mkdir -p $O
for i in 1 2; do
  for m in bert resnet50; do
    (cd $R/ab_prev && timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 2>/dev/null > $O/b.json) || exit 1
    echo "prev $m $(cut -c1-140 $O/b.json)" | tee -a $O/bench.txt
    timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 2>/dev/null > $O/b.json || exit 1
    echo "head $m $(cut -c1-140 $O/b.json)" | tee -a $O/bench.txt
  done
done
