#!/bin/bash
# Third GPU call: four-wave weight gradients, the GEMM knob sweep, ResNet-50 with the four-wave routing.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
fatal() { case $1 in 124|134|137|139) echo "[batch3] fatal rc=$1 in $2"; exit $1;; esac; }
bash scripts/r4/w4_wgrad.sh; rc=$?; echo "[batch3] w4_wgrad rc=$rc"; fatal $rc w4_wgrad
for v in 0 1; do
  DDL_GEMM_W4=$v timeout -k 10 300 python bench.py --steps 15 --warmup 4 > gpurun_out/r4/bench_rn50_w4_$v.json 2> gpurun_out/r4/bench_rn50_w4_$v.err
  rc=$?; echo "[batch3] rn50 w4=$v rc=$rc"; cat gpurun_out/r4/bench_rn50_w4_$v.json; fatal $rc rn50
done
bash scripts/r4/gemm_sweep.sh; rc=$?; echo "[batch3] gemm_sweep rc=$rc"
exit 0
