#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 120 python scripts/r5/mnist_step.py > gpurun_out/r5/mnist_step.log 2>&1 || { cat gpurun_out/r5/mnist_step.log; exit 1; }
cat gpurun_out/r5/mnist_step.log | grep -v amdgpu.ids
REPS=100 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/step_prof -o step -- python scripts/r5/mnist_step.py > gpurun_out/r5/step_prof.log 2>&1
find gpurun_out/r5/step_prof -type f ! -name '*kernel_stats.csv' -delete
cd examples && timeout -k 10 240 python -u ddl_mnist.py --executors 4 --processes 2 --epochs 5 --train-rows 60000 --test-rows 10000 --workers-per-gpu 8 > ../gpurun_out/r5/mnist.log 2>&1
grep "Training time\|Accuracy\|updates" ../gpurun_out/r5/mnist.log
