#!/bin/bash
# Replica-batched Sequential CNN: the batched-vs-stream test, the 8-worker MNIST example, then the grad-norm spread.
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_colocated.py -k "cnn or capture" > gpurun_out/r5/t_seq.log 2>&1 || { echo TESTS FAILED; grep -E "Error|^E " gpurun_out/r5/t_seq.log | head -30; exit 1; }
tail -2 gpurun_out/r5/t_seq.log
cd examples && timeout -k 10 240 python -u ddl_mnist.py --executors 4 --processes 2 --epochs 5 --train-rows 60000 --test-rows 10000 --workers-per-gpu 8 > ../gpurun_out/r5/mnist_seq.log 2>&1 || { tail -30 ../gpurun_out/r5/mnist_seq.log; exit 1; }
grep "Training time\|Accuracy\|updates" ../gpurun_out/r5/mnist_seq.log
cd .. && timeout -k 10 500 python scripts/r5/gradnorm_spread.py > gpurun_out/r5/gradnorm_spread.txt 2>&1
