#!/bin/bash
# Gathered weight-gradient split-K rounds x tile sweep on the ResNet-50 per-layer table
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/wsweep; mkdir -p $O
for t in auto 128; do
  for r in 1 2 4; do
    DDL_WGRAD_TILE=$t DDL_WGRAD_ROUNDS=$r timeout -k 10 300 python scripts/bench_resnet_layers.py > $O/l_${t}_$r.json 2>/dev/null || exit 1
    echo "tile=$t rounds=$r $(python -c "import json;d=json.load(open('$O/l_${t}_$r.json'));print(d['total_ms_per_step'])")"
  done
done
