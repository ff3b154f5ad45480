#!/bin/bash
# Round 4 baseline on one MI355X: headline benches + GEMM microbenchmark at HEAD.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4/bench_resnet.log 2>&1 || { tail -20 gpurun_out/r4/bench_resnet.log; exit 1; }
grep '^{' gpurun_out/r4/bench_resnet.log
timeout -k 10 300 python bench.py --model bert --steps 10 --warmup 3 > gpurun_out/r4/bench_bert.log 2>&1 || { tail -20 gpurun_out/r4/bench_bert.log; exit 1; }
grep '^{' gpurun_out/r4/bench_bert.log
timeout -k 10 300 python bench.py --model vgg16 --steps 20 --warmup 5 > gpurun_out/r4/bench_vgg.log 2>&1 || { tail -20 gpurun_out/r4/bench_vgg.log; exit 1; }
grep '^{' gpurun_out/r4/bench_vgg.log
timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/r4/gemm_micro.jsonl 2>&1 || { tail -20 gpurun_out/r4/gemm_micro.jsonl; exit 1; }
cat gpurun_out/r4/gemm_micro.jsonl
