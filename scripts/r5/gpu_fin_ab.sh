#!/bin/bash
# BN finalize operand prefetch: BN tests, then same-box ResNet-50 A/B against ab/base (HEAD before the change).
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_stem.py \
  -k "bn or stem or bottleneck" > gpurun_out/r5/fin_tests.log 2>&1 || { tail -30 gpurun_out/r5/fin_tests.log; exit 1; }
tail -1 gpurun_out/r5/fin_tests.log
ROUNDS=3 TAG=${TAG:-fin_ab} bash scripts/r5/ab.sh || exit 1
