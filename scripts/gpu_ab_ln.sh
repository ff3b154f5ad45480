#!/bin/bash
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/ab_ln; mkdir -p $O
for r in 1 2 3; do
  for v in 0 1; do
    DDL_LN_FWD_WAVE_ROWS=$v timeout -k 10 300 python bench.py --model bert --steps 10 --warmup 3 > $O/b_${v}_$r.log 2>&1 || exit 1
    echo "wave_rows=$v r$r $(tail -1 $O/b_${v}_$r.log | grep -o '"value": [0-9.]*')"
  done
done
