#!/bin/bash
# Graph-replayed dropout: tests, VGG-16 host/device split, VGG-16 eager vs graph (interleaved, 3 rounds).
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 200 python -u -m pytest tests/test_gpu_graph_dropout.py tests/test_gpu_graphs.py -x -v --timeout 100 \
  --timeout-method thread > gpurun_out/r6/graph_dropout.log 2>&1 || { tail -30 gpurun_out/r6/graph_dropout.log; exit 1; }
timeout -k 10 300 python -u scripts/r6/host_device_split.py vgg16 > gpurun_out/r6/host_device_vgg.jsonl 2>&1 || exit 1
out=gpurun_out/r6/ab_vgg_graph.txt
: > $out
for r in 1 2 3; do
  for g in 0 1; do
    timeout -k 10 200 python -u bench.py --model vgg16 --steps 50 --warmup 10 --graph $g 2>/dev/null \
      | sed "s/^/vgg16 graph=$g /" >> $out || exit 1
  done
done
