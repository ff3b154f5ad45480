#!/bin/bash
# Same-box A/B of the VGG-16 fusions (conv-BN-ReLU-pool node; BN reduce in the next conv's dgrad epilogue).
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_layers.py tests/test_gpu_kernels.py \
  -k "chain or pool or sequential" > gpurun_out/r5/vgg_ab_tests.log 2>&1 || { tail -30 gpurun_out/r5/vgg_ab_tests.log; exit 1; }
tail -1 gpurun_out/r5/vgg_ab_tests.log
SWITCH="distributeddeeplearningspark_amd.ops.fused_blocks:_SEQ_POOL=False" ARGS="--model vgg16" ROUNDS=4 TAG=vgg_ab/pool bash scripts/r5/ab_toggle.sh || exit 1
SWITCH="distributeddeeplearningspark_amd.ops.fused_blocks:_FUSE_BNR=False" ARGS="--model vgg16" ROUNDS=4 TAG=vgg_ab/bnr bash scripts/r5/ab_toggle.sh || exit 1
