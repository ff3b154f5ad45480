#!/bin/bash
# 3x3 weight-gradient halo kernel, round 2: tests (2-block / ping-pong, atomics / slabs), per-shape
# microbenchmark with kernel stats, interleaved ResNet-50 A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "wgrad_halo or resnet50_step or per_layer" > gpurun_out/wg3b_tests.log 2>&1
rc=$?; tail -3 gpurun_out/wg3b_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error" gpurun_out/wg3b_tests.log | head -20; exit $rc; }
timeout -k 10 300 python scripts/bench_wgrad3.py > gpurun_out/wg3b_micro.jsonl 2>&1 || { tail -20 gpurun_out/wg3b_micro.jsonl; exit 1; }
cat gpurun_out/wg3b_micro.jsonl
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/wg3b_mprof -- python3 $GRAFT_REPO_ROOT/scripts/bench_wgrad3.py > $GRAFT_REPO_ROOT/gpurun_out/wg3b_mprof.log 2>&1 ) || { echo "rocprof failed"; exit 1; }
f=$(find gpurun_out/wg3b_mprof -name "*kernel_stats.csv" | head -1)
python scripts/prof_summary.py $f 1 gpurun_out/wg3b_micro_kstats.csv | grep -E "wgrad|gemm_dma" | head -30
OUT=gpurun_out/ab_wg3b.jsonl; : > $OUT
for r in 1 2; do
  for cfg in "DDL_WGRAD3X3_PP=0" "DDL_WGRAD3X3_PP=1" "DDL_WGRAD3X3=0"; do
    env $cfg timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/ab_tmp.log 2>&1 || { echo "bench $cfg failed"; tail -20 gpurun_out/ab_tmp.log; exit 1; }
    line=$(grep '^{' gpurun_out/ab_tmp.log | tail -1)
    echo "{\"round\": $r, \"cfg\": \"$cfg\", \"bench\": $line}" >> $OUT
    echo "r$r $cfg $(echo $line | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
  done
done
