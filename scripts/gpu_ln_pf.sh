#!/bin/bash
# After the 16-B parameter loads in the LayerNorm / BN-reduce kernels: full GPU suite, LN and BN
# microbenches, BERT-base and ResNet-50 benches.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/lnpf; mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python scripts/bench_layernorm.py || exit 1
timeout -k 10 200 python scripts/bench_bn.py > $O/bn.txt 2>&1 || exit 1
grep "{" $O/bn.txt
for r in 1 2; do
  for m in bert resnet50; do
    timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > $O/${m}_$r.log 2>&1 || { tail $O/${m}_$r.log; exit 1; }
    echo "$m r$r $(tail -1 $O/${m}_$r.log | grep -o '"value": [0-9.]*')"
  done
done
