#!/bin/bash
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/wsweep; mkdir -p $O
for r in 6 8; do
  DDL_WGRAD_ROUNDS=$r timeout -k 10 300 python scripts/bench_resnet_layers.py > $O/l_auto_$r.json 2>/dev/null || exit 1
  echo "rounds=$r $(python -c "import json;d=json.load(open('$O/l_auto_$r.json'));print(d['total_ms_per_step'])")"
done
export TMPDIR=/tmp
R=$(pwd)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_vgg2 -- python3 $R/bench.py --model vgg16 --steps 5 --warmup 2 > $R/gpurun_out/prof_vgg2.log 2>&1
echo "rocprof rc=$?"
