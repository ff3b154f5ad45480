#!/bin/bash
# Early (begin_step, side stream) derived-filter batch: test, same-box BERT-base A/B; then end-of-round part 2.
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_layers.py \
  -k "derived or taps" > gpurun_out/r5/early_tests.log 2>&1 || { tail -30 gpurun_out/r5/early_tests.log; exit 1; }
tail -1 gpurun_out/r5/early_tests.log
SWITCH="distributeddeeplearningspark_amd.ops.derived:EARLY=False" ARGS="--model bert --steps 10 --warmup 3" ROUNDS=3 TAG=early_ab/bert bash scripts/r5/ab_toggle.sh || exit 1
bash scripts/r5/gpu_final2.sh
