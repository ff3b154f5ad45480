#!/bin/bash
# 64-channel 3x3 resident-filter kernel (pipelined, deferred epilogue): tests, microbench, PMC, ResNet A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "c64 or halo_kernel" > gpurun_out/c64_tests.log 2>&1
rc=$?; tail -2 gpurun_out/c64_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error" gpurun_out/c64_tests.log | head -20; exit $rc; }
: > gpurun_out/c64_micro.jsonl
for v in 1 0; do
  DDL_CONV3X3_C64PP=$v timeout -k 10 200 python scripts/bench_c64.py >> gpurun_out/c64_micro.jsonl 2>&1 || { tail gpurun_out/c64_micro.jsonl; exit 1; }
done
grep '^{' gpurun_out/c64_micro.jsonl
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmc_c64; mkdir -p $O
( cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -- python3 $R/scripts/bench_c64.py > $O/trace.log 2>&1 ) || { echo trace failed; exit 1; }
( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES --output-format csv -d $O/p1 -- python3 $R/scripts/bench_c64.py > $O/p1.log 2>&1 ) || { echo p1 failed; exit 1; }
( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/p2 -- python3 $R/scripts/bench_c64.py > $O/p2.log 2>&1 ) || { echo p2 failed; exit 1; }
t=$(find $O/trace -name "*kernel_trace.csv" | head -1); a=$(find $O/p1 -name "*counter_collection.csv" | head -1); b=$(find $O/p2 -name "*counter_collection.csv" | head -1)
python scripts/pmc_table.py $t $a $b > gpurun_out/pmc_c64_table.txt 2>&1; grep -E "kernel|c64|gemm_dma" gpurun_out/pmc_c64_table.txt | head -12
OUT=gpurun_out/ab_c64.jsonl; : > $OUT
for r in 1 2; do
  for cfg in "DDL_CONV3X3_C64PP=1" "DDL_CONV3X3_C64PP=0"; do  # (Python gate: opt-in with =1)
    env $cfg timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/ab_tmp.log 2>&1 || { echo "bench $cfg failed"; tail -20 gpurun_out/ab_tmp.log; exit 1; }
    line=$(grep '^{' gpurun_out/ab_tmp.log | tail -1)
    echo "{\"round\": $r, \"cfg\": \"$cfg\", \"bench\": $line}" >> $OUT
    echo "r$r $cfg $(echo $line | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
  done
done
