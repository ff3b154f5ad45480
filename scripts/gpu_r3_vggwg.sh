#!/bin/bash
# VGG-16 3x3 weight gradients of the 8 / 4 / 2 pixel blocks on the halo kernel: numerics, the ResNet-50
# step test under both BN store forms, interleaved VGG-16 A/B (DDL_WGRAD3X3=0: gathered GEMM), profile
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_layers.py -k "wgrad_halo or sequential_fused or vgg" > gpurun_out/vggwg_tests.log 2>&1
rc=$?; tail -1 gpurun_out/vggwg_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/vggwg_tests.log | head -20; exit $rc; }
for v in 0 1; do
  DDL_BN_NT=$v timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k test_resnet50_step_matches_reference > gpurun_out/vggwg_nt$v.log 2>&1
  echo "resnet50 step test NT=$v: $(tail -1 gpurun_out/vggwg_nt$v.log)"; grep -E "^E.*cpu" gpurun_out/vggwg_nt$v.log | head -2
done
OUT=gpurun_out/ab_vggwg.jsonl; : > $OUT
for r in 1 2 3; do
  for v in 1 0; do
    DDL_WGRAD3X3=$v timeout -k 10 300 python bench.py --model vgg16 --steps 50 --warmup 10 > gpurun_out/ab_tmp.log 2>&1 || { tail gpurun_out/ab_tmp.log; exit 1; }
    line=$(grep '^{' gpurun_out/ab_tmp.log | tail -1)
    echo "{\"round\": $r, \"model\": \"vgg16\", \"DDL_WGRAD3X3\": \"$v\", \"bench\": $line}" >> $OUT
    echo "r$r vgg16 wg3=$v $(echo $line | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
  done
done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/vggwg_prof -- python3 $GRAFT_REPO_ROOT/bench.py --model vgg16 --steps 10 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/vggwg_prof.log 2>&1 ) || { echo "rocprof failed"; tail -20 gpurun_out/vggwg_prof.log; exit 1; }
f=$(find gpurun_out/vggwg_prof -name "*kernel_stats.csv" | head -1)
python scripts/prof_summary.py $f 15 gpurun_out/vggwg_kstats.csv | head -16
