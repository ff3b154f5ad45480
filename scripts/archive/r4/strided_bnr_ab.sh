#!/bin/bash
# A/B of the strided-class BN reduce (DDL_STRIDED_BNR 0 / 1) after the whole-wave statistics atomics, interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r4/strided_bnr2; mkdir -p $O
for i in 1 2 3; do
  for v in 0 1; do
    DDL_STRIDED_BNR=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 2>/dev/null > $O/b.json || exit 1
    echo "strided_bnr=$v $(cut -c1-150 $O/b.json)" | tee -a $O/bench.txt
  done
done
for m in bert vgg16; do
  timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 2>/dev/null > $O/b.json || exit 1
  echo "$m $(cut -c1-150 $O/b.json)" | tee -a $O/bench.txt
done
