#!/bin/bash
# Round 3: co-located worker workflows (MNIST 8 workers, NYISO GRU/LSTM 4 workers) on one GPU.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_colocated.py -x -v --timeout 300 --timeout-method thread > gpurun_out/colocated_tests.log 2>&1
rc=$?; tail -5 gpurun_out/colocated_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python examples/ddl_mnist.py --executors 4 --processes 2 --epochs 5 --train-rows 60000 --test-rows 10000 --workers-per-gpu 8 > gpurun_out/mnist_8workers.log 2>&1 || { tail -30 gpurun_out/mnist_8workers.log; exit 1; }
grep -E "Training time|Accuracy|updates|Workers" gpurun_out/mnist_8workers.log
for m in nyiso_gru nyiso_lstm; do
  timeout -k 10 400 python bench.py --model $m > gpurun_out/bench_$m.json 2> gpurun_out/bench_$m.err || { tail -30 gpurun_out/bench_$m.err; exit 1; }
  cat gpurun_out/bench_$m.json
done
if [ "${VGG_OVERHEAD:-1}" = "1" ]; then
  timeout -k 10 200 python scripts/cpu_overhead.py --model vgg16 --steps 30 > gpurun_out/cpu_overhead_vgg.txt 2>&1 || exit 1
  head -3 gpurun_out/cpu_overhead_vgg.txt
fi
