#!/bin/bash
# MNIST ADAG workflow (8 co-located workers, 60k rows, 5 epochs; and 1 worker) with the per-worker
# breakdown; A/B against a worktree of an older commit when AB_OLD names one (same box, interleaved).
set -u
cd "$(dirname "$0")/.."
R=$(pwd)
O=$R/gpurun_out/ab; mkdir -p $O
for t in . ${AB_OLD:-}; do
  n=$(basename $t)
  (cd $t && timeout -k 10 300 python examples/ddl_mnist.py --executors 4 --processes 2 --epochs 5 --train-rows 60000 --test-rows 10000 --workers-per-gpu 8 > $O/mnist8_$n.log 2>&1) || exit 1
  echo "8 workers $t $(grep 'Training time' $O/mnist8_$n.log)"; grep Workers $O/mnist8_$n.log | cut -c1-400
  (cd $t && timeout -k 10 300 python examples/ddl_mnist.py --executors 1 --processes 1 --epochs 1 --train-rows 16000 --test-rows 1000 > $O/mnist1_$n.log 2>&1) || exit 1
  echo "1 worker $t $(grep 'Training time' $O/mnist1_$n.log)"; grep Workers $O/mnist1_$n.log
done
for m in nyiso_gru nyiso_lstm; do
  timeout -k 10 300 python bench.py --model $m > $O/$m.json 2> $O/$m.log || exit 1
  tail -1 $O/$m.json | cut -c1-200
done
