#!/bin/bash
# One-launch parity-class strided data-gradients: tests, per-layer roofline, same-box ResNet-50 A/B.
export TMPDIR=/tmp
O=gpurun_out/r5/zcls
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "strided_dgrad_classes or conv_fwd_bwd or bottleneck or resnet or dgrad" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python scripts/bench_resnet_layers.py > $O/resnet50_layer_roofline.json 2> $O/roof.err || exit 1
SWITCH="distributeddeeplearningspark_amd.ops.conv:_CLASS_BATCH=False" ROUNDS=3 TAG=zcls/ab bash scripts/r5/ab_toggle.sh || exit 1
