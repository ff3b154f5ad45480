#!/bin/bash
# Round-6 HEAD baseline on one MI355X: smoke, ResNet-50 bench x2, BERT-base bench x1.
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6/smoke.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6/bench_rn50.jsonl 2>gpurun_out/r6/bench_rn50.err &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 >> gpurun_out/r6/bench_rn50.jsonl 2>>gpurun_out/r6/bench_rn50.err &&
timeout -k 10 200 python -u bench.py --model bert --steps 10 --warmup 3 > gpurun_out/r6/bench_bert.jsonl 2>gpurun_out/r6/bench_bert.err
