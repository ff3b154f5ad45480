#!/bin/bash
# The reference's own workloads on one MI355X: NYISO GRU/LSTM (ADAG, 4 workers co-located)
# and the MNIST CNN (ADAG, 8 workers co-located, batch 16, window 5).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 ${T:-300} python -u -m pytest tests/test_gpu_graphs.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/graphs_tests.log 2>&1
rc=$?; tail -n 8 gpurun_out/graphs_tests.log
if [ $rc -ne 0 ]; then echo "graph tests rc=$rc"; exit $rc; fi
timeout -k 10 400 python -u examples/ddl_nyiso.py --workers 4 --workers-per-gpu 4 --epochs 20 > gpurun_out/nyiso4.log 2>&1 || exit $?
tail -n 1 gpurun_out/nyiso4.log
timeout -k 10 600 python -u examples/ddl_mnist.py --executors 4 --processes 2 --workers-per-gpu 8 --epochs ${MNIST_EPOCHS:-5} --train-rows ${MNIST_ROWS:-60000} --test-rows 10000 > gpurun_out/mnist8.log 2>&1 || exit $?
tail -n 4 gpurun_out/mnist8.log
