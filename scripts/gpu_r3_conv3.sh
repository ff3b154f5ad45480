#!/bin/bash
# convolution kernel-knob A/B (one process per variant, interleaved twice)
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/conv3_var2.jsonl
: > $OUT
for r in 1 2; do
  timeout -k 10 120 python scripts/bench_conv3x3_var.py base >> $OUT || exit 1
  DDL_WGRAD_ROUNDS=1 DDL_LINEAR_WGRAD_ROUNDS=0.5 timeout -k 10 120 python scripts/bench_conv3x3_var.py r1 >> $OUT || exit 1
  DDL_WGRAD_ROUNDS=2 timeout -k 10 120 python scripts/bench_conv3x3_var.py r2 >> $OUT || exit 1
  DDL_WGRAD_ROUNDS=1 DDL_GATHER_STAGES=3 DDL_LINEAR_WGRAD_ROUNDS=0.5 timeout -k 10 120 python scripts/bench_conv3x3_var.py r1st3 >> $OUT || exit 1
  DDL_WGRAD_ROUNDS=2 DDL_GATHER_STAGES=3 timeout -k 10 120 python scripts/bench_conv3x3_var.py r2st3 >> $OUT || exit 1
done
