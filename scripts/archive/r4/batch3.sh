#!/bin/bash
# GEMM knob sweep (ring / double-stage LDS for the 128x128 kernel, split-K slabs), attention occupancy on
# the whole BERT step.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
fatal() { case $1 in 124|134|137|139) echo "[batch3] fatal rc=$1 in $2"; exit $1;; esac; }
bash scripts/r4/gemm_sweep.sh; rc=$?; echo "[batch3] gemm_sweep rc=$rc"; fatal $rc sweep
for v in 2 3; do
  DDL_ATTN_FWD_OCC=$v timeout -k 10 300 python bench.py --model bert --steps 10 --warmup 3 > gpurun_out/r4/bench_bert_fwdocc_$v.json 2>/dev/null
  rc=$?; echo "[batch3] bert fwd_occ=$v rc=$rc"; cat gpurun_out/r4/bench_bert_fwdocc_$v.json; fatal $rc bert
done
exit 0
