#!/bin/bash
# vectorised softmax cross-entropy: loss tests + BERT bench
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/xent; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_transformer.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --model bert --steps 10 --warmup 3 > $O/bert_$r.log 2>&1 || { tail $O/bert_$r.log; exit 1; }
  echo "bert r$r $(tail -1 $O/bert_$r.log | grep -o '"value": [0-9.]*')"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OLDPWD/$O/prof -- python3 $OLDPWD/bench.py --model bert --steps 3 --warmup 1 > $OLDPWD/$O/prof.log 2>&1 || { echo "prof failed"; exit 1; }
cd $OLDPWD; f=$(ls $O/prof/*/*_kernel_stats.csv | head -1); grep -i "xent" $f | cut -c1-160
