#!/bin/bash
# Row-tap gathers for the s2d stem: tests, same-box ResNet-50 A/B.
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stem.py tests/test_gpu_kernels.py \
  -k "stem or conv_fwd_bwd or gemm" > gpurun_out/r5/rowtap_tests.log 2>&1 || { tail -30 gpurun_out/r5/rowtap_tests.log; exit 1; }
tail -1 gpurun_out/r5/rowtap_tests.log
SWITCH="distributeddeeplearningspark_amd.ops.fused_blocks:_STEM_ROWTAP=False" ROUNDS=3 TAG=rowtap_ab bash scripts/r5/ab_toggle.sh || exit 1
