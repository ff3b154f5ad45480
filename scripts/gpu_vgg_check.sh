#!/bin/bash
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/vggc; mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python bench.py --model vgg16 --steps 30 --warmup 5 > $O/vgg_$r.log 2>&1 || exit 1
  echo "vgg r$r $(tail -1 $O/vgg_$r.log | cut -c55-100)"
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/rn_$r.log 2>&1 || exit 1
  echo "rn r$r $(tail -1 $O/rn_$r.log | cut -c80-120)"
done
R=$(pwd); cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_vgg3 -- python3 $R/bench.py --model vgg16 --steps 5 --warmup 2 > $R/gpurun_out/prof_vgg3.log 2>&1
echo "rocprof rc=$?"
