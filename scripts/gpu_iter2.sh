#!/bin/bash
# quick iteration + VGG + gathered ring depth A/B (layer table + benches)
set -u
cd "$(dirname "$0")/.."
bash scripts/gpu_quick.sh || exit 1
O=gpurun_out/iter2; mkdir -p $O
timeout -k 10 300 python bench.py --model vgg16 --steps 20 --warmup 5 > $O/vgg.log 2>&1 || exit 1
echo "vgg $(tail -1 $O/vgg.log | cut -c55-100)"
for st in 3 4; do
  DDL_GATHER_STAGES=$st timeout -k 10 300 python scripts/bench_resnet_layers.py > $O/layers_g$st.json 2>/dev/null || exit 1
  echo "gather stages=$st $(python -c "import json;d=json.load(open('$O/layers_g$st.json'));print(d['total_ms_per_step'])")"
  DDL_GATHER_STAGES=$st timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/rn_g$st.log 2>&1 || exit 1
  echo "  rn $(tail -1 $O/rn_g$st.log | cut -c80-120)"
  DDL_GATHER_STAGES=$st timeout -k 10 300 python bench.py --model vgg16 --steps 20 --warmup 5 > $O/vgg_g$st.log 2>&1 || exit 1
  echo "  vgg $(tail -1 $O/vgg_g$st.log | cut -c55-100)"
done
python -c "import json;d=json.load(open('gpurun_out/quick/layers.json'));print('default layers', d['total_ms_per_step'])"
