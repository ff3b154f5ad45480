#!/bin/bash
# Ring depth of the gathered fp32 kernels (conv wgrad, split-K forward): VGG-16 and ResNet-50
# benches and the ResNet per-layer table at DDL_GATHER_STAGES = 1 / 3 / 4.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/stages; mkdir -p $O
for st in 1 3 4; do
  DDL_GATHER_STAGES=$st timeout -k 10 300 python bench.py --model vgg16 --steps 20 --warmup 5 > $O/vgg_$st.log 2>&1 || exit 1
  DDL_GATHER_STAGES=$st timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/rn_$st.log 2>&1 || exit 1
  DDL_GATHER_STAGES=$st timeout -k 10 300 python scripts/bench_resnet_layers.py > $O/layers_$st.json 2> /dev/null || exit 1
  echo "st=$st vgg $(tail -1 $O/vgg_$st.log | cut -c60-100) rn $(tail -1 $O/rn_$st.log | cut -c80-120)"
done
