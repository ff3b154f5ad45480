#!/bin/bash
# MNIST workflow (examples/ddl_mnist.py) on the reference's 59,999 training rows (ragged shards): 8 co-located
# workers (4 executors x 2 processes) and 16 (8 x 2), 5 epochs, both expected on the batched replica path.
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u examples/ddl_mnist.py --executors 4 --processes 2 --epochs 5 --train-rows 59999 \
  --workers-per-gpu 8 > gpurun_out/r6/mnist_8w_59999.txt 2>&1 &&
timeout -k 10 300 python -u examples/ddl_mnist.py --executors 8 --processes 2 --epochs 5 --train-rows 59999 \
  --workers-per-gpu 16 > gpurun_out/r6/mnist_16w_59999.txt 2>&1
