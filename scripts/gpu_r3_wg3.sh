#!/bin/bash
# 3x3 weight-gradient halo kernel: numerics tests, then an interleaved ResNet-50 A/B of its knobs
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "wgrad_halo or conv_fwd_bwd or resnet50_step or per_layer or bottleneck" > gpurun_out/wg3_tests.log 2>&1
rc=$?; tail -5 gpurun_out/wg3_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error" gpurun_out/wg3_tests.log | head -20; exit $rc; }
OUT=gpurun_out/ab_wg3.jsonl; : > $OUT
for r in 1 2; do
  for cfg in "DDL_WGRAD3X3=1" "DDL_WGRAD3X3=0" "DDL_WGRAD3X3_SLAB=1" "DDL_WGRAD3X3_BPC=1" "DDL_WGRAD3X3_BPC=1 DDL_WGRAD3X3_SLAB=1"; do
    env $cfg timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/ab_tmp.log 2>&1 || { echo "bench $cfg failed"; tail -20 gpurun_out/ab_tmp.log; exit 1; }
    line=$(grep '^{' gpurun_out/ab_tmp.log | tail -1)
    echo "{\"round\": $r, \"cfg\": \"$cfg\", \"bench\": $line}" >> $OUT
    echo "r$r $cfg $(echo $line | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
  done
done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/wg3_prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/wg3_prof.log 2>&1 ) || { echo "rocprof failed"; tail -20 gpurun_out/wg3_prof.log; exit 1; }
f=$(find gpurun_out/wg3_prof -name "*kernel_stats.csv" | head -1)
python scripts/prof_summary.py $f 7 gpurun_out/wg3_kstats.csv | head -30
