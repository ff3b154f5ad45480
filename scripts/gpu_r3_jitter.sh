#!/bin/bash
# VGG-16 step jitter (per-step GPU / host time percentiles), 3 runs, with a clock snapshot
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
(rocm-smi --showclocks 2>/dev/null | grep -E "sclk|mclk" | head -4) || true
for i in 1 2 3; do
  timeout -k 10 200 python scripts/vgg_jitter.py 200 2>&1 | grep '^{' | tee -a gpurun_out/vgg_jitter.jsonl || exit 1
done
(rocm-smi --showclocks 2>/dev/null | grep -E "sclk|mclk" | head -4) || true
