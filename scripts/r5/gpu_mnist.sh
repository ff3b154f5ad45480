#!/bin/bash
# GPU check of the MNIST launch diet: layer tests, the 8-worker example, the per-step op list.
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_layers.py tests/test_gpu_colocated.py > gpurun_out/r5/t_mnist.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r5/t_mnist.log; exit 1; }
tail -3 gpurun_out/r5/t_mnist.log
timeout -k 10 200 python scripts/r5/mnist_ops.py > gpurun_out/r5/mnist_ops.txt 2>&1 || exit 1
cd examples && timeout -k 10 240 python -u ddl_mnist.py --executors 4 --processes 2 --epochs 5 --train-rows 60000 --test-rows 10000 --workers-per-gpu 8 > ../gpurun_out/r5/mnist.log 2>&1
grep "Training time\|Accuracy\|updates" ../gpurun_out/r5/mnist.log
