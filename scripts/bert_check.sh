#!/bin/bash
# transformer kernel tests -> attention microbench -> BERT bench; stop on crash/timeout.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_transformer.py -x -q > gpurun_out/tr_tests.log 2>&1
rc=$?
tail -3 gpurun_out/tr_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
timeout -k 10 200 python scripts/bench_attention.py > gpurun_out/bench_attn.log 2>&1 || exit $?
grep drop gpurun_out/bench_attn.log
timeout -k 10 400 python bench.py --model bert --steps 5 --warmup 2 > gpurun_out/bench_bert.log 2>&1 || exit $?
tail -1 gpurun_out/bench_bert.log | cut -c1-220
exit $rc
