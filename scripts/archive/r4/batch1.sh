#!/bin/bash
# One GPU call: attention rebuild + dropout hash, four-wave GEMM, BERT-base step with and without the new
# GEMM routing.  A step that fails its checks is reported and the next one runs; a fault / abort / time
# limit ends the call.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
fatal() { case $1 in 124|134|137|139) echo "[batch1] fatal rc=$1 in $2"; exit $1;; esac; }
bash scripts/r4/attn.sh; rc=$?; echo "[batch1] attn.sh rc=$rc"; fatal $rc attn
bash scripts/r4/w4.sh; rc=$?; echo "[batch1] w4.sh rc=$rc"; fatal $rc w4
for v in 0 1 2; do
  DDL_GEMM_W4=$v timeout -k 10 300 python bench.py --model bert --steps 10 --warmup 3 > gpurun_out/r4/bench_bert_w4_$v.json 2> gpurun_out/r4/bench_bert_w4_$v.err
  rc=$?; echo "[batch1] bert w4=$v rc=$rc"; cat gpurun_out/r4/bench_bert_w4_$v.json; fatal $rc bert_w4
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r4/bench_rn50.json 2> gpurun_out/r4/bench_rn50.err
rc=$?; echo "[batch1] rn50 rc=$rc"; cat gpurun_out/r4/bench_rn50.json
exit 0
