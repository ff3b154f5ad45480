#!/bin/bash
# stem + transformer kernel tests -> attention microbench -> BERT and ResNet-50 benches.
# Each GPU step has its own time limit; any crash/timeout ends the script.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -2 "gpurun_out/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "[$name] rc=$rc"; exit $rc; fi
}
step stem_tests 300 python -m pytest tests/test_gpu_stem.py -x -q
step tr_tests 300 python -m pytest tests/test_gpu_transformer.py -x -q
step bench_attn 200 python scripts/bench_attention.py
step bench_bert 400 python bench.py --model bert --steps 10 --warmup 3
step bench_resnet 400 python bench.py --steps 10 --warmup 3
