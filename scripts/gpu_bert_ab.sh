#!/bin/bash
# BERT-base A/B: default vs DDL_WGRAD_STAGES=1 (single-stage weight-gradient kernels), interleaved
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/bert_ab; mkdir -p $O
for r in 1 2; do
  for v in default 1; do
    if [ $v = default ]; then E=""; else E="DDL_WGRAD_STAGES=$v"; fi
    env $E timeout -k 10 300 python bench.py --model bert --steps 10 --warmup 3 > $O/bert_${v}_$r.log 2>&1 || exit 1
    echo "$v r$r $(tail -1 $O/bert_${v}_$r.log | cut -c60-100)"
  done
done
