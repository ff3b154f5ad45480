#!/bin/bash
# VGG-16 (CIFAR shape, batch 256) kernel profile at HEAD, summarised by scripts/r5/trace_busy.py.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6/prof2
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/vgg -o vgg -- python3 $R/bench.py --model vgg16 --steps 20 --warmup 5 > $O/vgg.log 2>&1 || exit 1
python3 $R/scripts/r5/trace_busy.py $(find $O/vgg -name '*kernel_trace.csv') 40 > $O/vgg_busy.txt || exit 1
find $O -type f -name '*kernel_trace.csv' -delete
