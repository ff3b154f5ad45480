#!/bin/bash
# VGG-16 and BERT-base benches plus a VGG kernel profile (after the ResNet quick iteration).
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/models; mkdir -p $O
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 300 python bench.py --model vgg16 --steps 20 --warmup 5 > $O/vgg.log 2>&1 || { tail $O/vgg.log; exit 1; }
tail -1 $O/vgg.log | cut -c1-160
timeout -k 10 300 python bench.py --model bert --steps 10 --warmup 3 > $O/bert.log 2>&1 || { tail $O/bert.log; exit 1; }
tail -1 $O/bert.log | cut -c1-160
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_vgg -- python3 $R/bench.py --model vgg16 --steps 5 --warmup 2 > $R/gpurun_out/prof_vgg.log 2>&1
echo "rocprof rc=$?"
