#!/bin/bash
# MNIST 8 co-located workers: per-kernel and HIP API statistics (rocprofv3), plus a busy-time summary.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
cd examples
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d ../gpurun_out/r5/mnist_prof -o mnist -- python -u ddl_mnist.py --executors 4 --processes 2 --epochs 5 --train-rows 60000 --test-rows 10000 --workers-per-gpu 8 > ../gpurun_out/r5/mnist_prof.log 2>&1
python ../scripts/r5/trace_busy.py $(find ../gpurun_out/r5/mnist_prof -name '*kernel_trace.csv') 40 > ../gpurun_out/r5/mnist_busy.txt
find ../gpurun_out/r5/mnist_prof -type f ! -name '*stats.csv' -delete
du -sh ../gpurun_out/r5/mnist_prof
