#!/bin/bash
# Round 4: in-process replica groups (parallel/replicas.py) on one MI355X — tests, then the
# reference workloads (MNIST 8 workers, NYISO GRU / LSTM 4 workers) vs the process-per-worker path.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_colocated.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r4/colocated_tests.log 2>&1
rc=$?; tail -12 gpurun_out/r4/colocated_tests.log
[ $rc -ne 0 ] && exit $rc
for m in nyiso_gru nyiso_lstm; do
  timeout -k 10 300 python bench.py --model $m > gpurun_out/r4/bench_${m}_groups.json 2> gpurun_out/r4/bench_${m}_groups.err || { tail -30 gpurun_out/r4/bench_${m}_groups.err; exit 1; }
  cat gpurun_out/r4/bench_${m}_groups.json
done
DDL_REPLICA_GROUPS=0 timeout -k 10 300 python bench.py --model nyiso_gru > gpurun_out/r4/bench_nyiso_gru_procs.json 2> gpurun_out/r4/bench_nyiso_gru_procs.err || { tail -30 gpurun_out/r4/bench_nyiso_gru_procs.err; exit 1; }
cat gpurun_out/r4/bench_nyiso_gru_procs.json
timeout -k 10 400 python examples/ddl_mnist.py --executors 4 --processes 2 --epochs 5 --train-rows 60000 --test-rows 10000 --workers-per-gpu 8 > gpurun_out/r4/mnist_8workers_groups.log 2>&1 || { tail -30 gpurun_out/r4/mnist_8workers_groups.log; exit 1; }
grep -E "Training time|Accuracy|updates|Workers" gpurun_out/r4/mnist_8workers_groups.log
