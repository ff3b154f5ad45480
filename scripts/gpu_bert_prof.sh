#!/bin/bash
set -u
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "conv or splitk" > gpurun_out/t_conv.log 2>&1 || { tail -20 gpurun_out/t_conv.log; exit 1; }
tail -1 gpurun_out/t_conv.log
timeout -k 10 300 python bench.py --model vgg16 --steps 30 --warmup 5 > gpurun_out/vgg_ws.log 2>&1 || exit 1
echo "vgg $(tail -1 gpurun_out/vgg_ws.log | cut -c55-100)"
R=$(pwd); cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bert2 -- python3 $R/bench.py --model bert --steps 5 --warmup 2 > $R/gpurun_out/prof_bert2.log 2>&1
echo "rocprof rc=$?"
