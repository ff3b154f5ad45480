#!/bin/bash
# BN apply / dx sweeps with 4 rows in flight per lane vs 2: numerics, sweep micro-bench, interleaved
# ResNet-50 A/B, then the VGG-16 kernel profile
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
DDL_BN_ROWS=4 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "batchnorm or bn_ or bottleneck" > gpurun_out/bnrows_tests.log 2>&1
rc=$?; tail -2 gpurun_out/bnrows_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/bnrows_tests.log | head -20; exit $rc; }
for v in 2 4 2nt 4nt; do
  nt=0; [ "${v#?}" = "nt" ] && nt=1
  DDL_BN_ROWS=${v:0:1} DDL_BN_NT=$nt timeout -k 10 120 python scripts/bench_bn.py > gpurun_out/bnrows_micro_$v.jsonl 2>gpurun_out/bnrows_micro.err || { tail gpurun_out/bnrows_micro.err; exit 1; }
  echo "rows=$v"; cut -c1-200 gpurun_out/bnrows_micro_$v.jsonl
done
OUT=gpurun_out/ab_bnrows.jsonl; : > $OUT
for r in 1 2; do
  for v in 4 2 4nt; do
    nt=0; [ "${v#?}" = "nt" ] && nt=1
    DDL_BN_ROWS=${v:0:1} DDL_BN_NT=$nt timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_tmp.log 2>&1 || { tail gpurun_out/ab_tmp.log; exit 1; }
    line=$(grep '^{' gpurun_out/ab_tmp.log | tail -1)
    echo "{\"round\": $r, \"DDL_BN_ROWS\": \"$v\", \"bench\": $line}" >> $OUT
    echo "r$r rows=$v $(echo $line | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
  done
done
bash scripts/gpu_r3_vggprof.sh
