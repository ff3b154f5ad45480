#!/bin/bash
# Vector path for tap-reordered filter copies: taps / derived / conv tests, same-box ResNet-50 A/B vs ab/base.
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_layers.py tests/test_gpu_kernels.py \
  -k "taps or derived or conv_fwd_bwd or strided or stride2" > gpurun_out/r5/taps_tests.log 2>&1 || { tail -30 gpurun_out/r5/taps_tests.log; exit 1; }
tail -1 gpurun_out/r5/taps_tests.log
ROUNDS=3 TAG=taps_ab bash scripts/r5/ab.sh || exit 1
