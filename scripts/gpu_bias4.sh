#!/bin/bash
# 16-B bias loads in the GEMM / streaming / split-K epilogues: full GPU suite + interleaved benches.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/bias4; mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python scripts/bench_epilogue.py > $O/epi.log 2>&1 || { tail $O/epi.log; exit 1; }
tail -12 $O/epi.log | cut -c1-200
for r in 1 2; do
  for m in bert resnet50 vgg16; do
    timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > $O/${m}_$r.log 2>&1 || { tail $O/${m}_$r.log; exit 1; }
    echo "$m r$r $(tail -1 $O/${m}_$r.log | grep -o '"value": [0-9.]*')"
  done
done
