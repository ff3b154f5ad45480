#!/bin/bash
# Per-layer gradient test, VGG-16 kernel profile, BERT-base bench.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/misc; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "per_layer or resnet50_step" > $O/tests.log 2>&1; rc=$?; tail -15 $O/tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --model vgg16 --steps 30 --warmup 5 > $O/vgg.log 2>&1 || exit 1
tail -1 $O/vgg.log
timeout -k 10 300 python bench.py --model bert --steps 10 --warmup 3 > $O/bert.log 2>&1 || exit 1
tail -1 $O/bert.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_vgg -- python3 $GRAFT_REPO_ROOT/bench.py --model vgg16 --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/$O/prof_vgg.log 2>&1
echo "rocprof rc=$?"
