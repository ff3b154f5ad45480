#!/bin/bash
# Interleaved A/B against the previous build in ab_prev/ (commit 514c1e2, before the whole-wave statistics
# atomics): BERT-base and ResNet-50 benches.
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
