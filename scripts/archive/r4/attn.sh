#!/bin/bash
# Attention rebuild (lazy running max, templated dropout / padding, 8-bit dropout bytes):
# correctness, micro-benchmark over the occupancy variants, BERT-base step.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_transformer.py -v --timeout 120 --timeout-method thread > gpurun_out/r4/attn_tests.log 2>&1
rc=$?; grep -E "FAIL|ERROR|passed|failed" gpurun_out/r4/attn_tests.log | tail -30
case $rc in 0|1) ;; *) exit $rc;; esac
: > gpurun_out/r4/attn_micro.txt
for v in "3 2 2" "4 2 3" "2 1 3"; do
  set -- $v
  echo "fwd_occ=$1 dkdv_occ=$2 dq_occ=$3" >> gpurun_out/r4/attn_micro.txt
  DDL_ATTN_FWD_OCC=$1 DDL_ATTN_DKDV_OCC=$2 DDL_ATTN_DQ_OCC=$3 timeout -k 10 120 python scripts/bench_attention.py >> gpurun_out/r4/attn_micro.txt 2>&1 || exit 1
done
cat gpurun_out/r4/attn_micro.txt
timeout -k 10 400 python bench.py --model bert --steps 10 --warmup 3 > gpurun_out/r4/bench_bert_attn.json 2> gpurun_out/r4/bench_bert_attn.err || { tail -30 gpurun_out/r4/bench_bert_attn.err; exit 1; }
cat gpurun_out/r4/bench_bert_attn.json
