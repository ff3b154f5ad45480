#!/bin/bash
# One GPU call: attention rebuild, four-wave GEMM, BERT-base step with and without the new GEMM routing.
# A step that fails its checks is reported and the next one runs; a fault / abort / time limit ends the call.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
fatal() { case $1 in 124|134|137|139) echo "[batch1] fatal rc=$1 in $2"; exit $1;; esac; }
bash scripts/r4/attn.sh; rc=$?; echo "[batch1] attn.sh rc=$rc"; fatal $rc attn
bash scripts/r4/w4.sh; rc=$?; echo "[batch1] w4.sh rc=$rc"; fatal $rc w4
DDL_GEMM_W4=1 timeout -k 10 300 python bench.py --model bert --steps 10 --warmup 3 > gpurun_out/r4/bench_bert_w4.json 2> gpurun_out/r4/bench_bert_w4.err
rc=$?; echo "[batch1] bert w4 rc=$rc"; cat gpurun_out/r4/bench_bert_w4.json; fatal $rc bert_w4
exit 0
