#!/bin/bash
# LayerNorm backward grid 2048 vs 1024 workgroups: transformer tests, same-box BERT-base A/B vs ab/base.
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_transformer.py \
  -k "layernorm or ln" > gpurun_out/r5/ln_tests.log 2>&1 || { tail -30 gpurun_out/r5/ln_tests.log; exit 1; }
tail -1 gpurun_out/r5/ln_tests.log
ARGS="--model bert --steps 10 --warmup 3" ROUNDS=3 TAG=ln_ab bash scripts/r5/ab.sh || exit 1
