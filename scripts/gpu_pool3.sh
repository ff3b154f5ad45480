#!/bin/bash
# stem max-pool backward on 2x2 input blocks: pool tests, microbench, ResNet-50 bench
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/pool3; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_layers.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python scripts/bench_pool.py 2>/dev/null || exit 1
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/rn_$r.log 2>&1 || { tail $O/rn_$r.log; exit 1; }
  echo "resnet50 r$r $(tail -1 $O/rn_$r.log | grep -o '"value": [0-9.]*')"
done
