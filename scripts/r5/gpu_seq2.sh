#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "resnet50_step_matches" tests/test_gpu_convergence.py -k "mnist or resnet50_step" > gpurun_out/r5/t_seq2.log 2>&1 || { echo TESTS FAILED; grep -E "Error|^E " gpurun_out/r5/t_seq2.log | head -30; exit 1; }
grep -E "PASSED|FAILED|ResNet-50 step|MNIST 8" gpurun_out/r5/t_seq2.log | cut -c1-250
cd examples && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ../gpurun_out/r5/mnist_seq_prof -o mnist -- python -u ddl_mnist.py --executors 4 --processes 2 --epochs 5 --train-rows 60000 --test-rows 10000 --workers-per-gpu 8 > ../gpurun_out/r5/mnist_seq_prof.log 2>&1
cd .. && python scripts/r5/trace_busy.py $(find gpurun_out/r5/mnist_seq_prof -name '*kernel_trace.csv') 40 > gpurun_out/r5/mnist_seq_busy.txt
find gpurun_out/r5/mnist_seq_prof -type f ! -name '*stats.csv' -delete
