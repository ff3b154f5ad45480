#!/bin/bash
# VGG-16 32x32 / 16x16 weight gradients on 128-pixel halo tiles: numerics, interleaved VGG-16 A/B
# (DDL_WGRAD3X3=0: gathered GEMM), ResNet-50 unchanged-tiling check + BN nontemporal-store A/B, profile
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_layers.py -k "wgrad_halo or sequential_fused or vgg or resnet" > gpurun_out/vggwg2_tests.log 2>&1
rc=$?; tail -1 gpurun_out/vggwg2_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/vggwg2_tests.log | head -20; exit $rc; }
OUT=gpurun_out/ab_vggwg2.jsonl; : > $OUT
for r in 1 2 3; do
  for v in 1 0; do
    DDL_WGRAD3X3=$v timeout -k 10 300 python bench.py --model vgg16 --steps 50 --warmup 10 > gpurun_out/ab_tmp.log 2>&1 || { tail gpurun_out/ab_tmp.log; exit 1; }
    line=$(grep '^{' gpurun_out/ab_tmp.log | tail -1)
    echo "{\"round\": $r, \"model\": \"vgg16\", \"DDL_WGRAD3X3\": \"$v\", \"bench\": $line}" >> $OUT
    echo "r$r vgg16 wg3=$v $(echo $line | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
  done
done
OUT=gpurun_out/ab_bnnt.jsonl; : > $OUT
for r in 1 2; do
  for v in 1 0; do
    DDL_BN_NT=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_tmp.log 2>&1 || { tail gpurun_out/ab_tmp.log; exit 1; }
    line=$(grep '^{' gpurun_out/ab_tmp.log | tail -1)
    echo "{\"round\": $r, \"model\": \"resnet50\", \"DDL_BN_NT\": \"$v\", \"bench\": $line}" >> $OUT
    echo "r$r resnet50 nt=$v $(echo $line | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
  done
done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/vggwg2_prof -- python3 $GRAFT_REPO_ROOT/bench.py --model vgg16 --steps 10 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/vggwg2_prof.log 2>&1 ) || { echo "rocprof failed"; tail -20 gpurun_out/vggwg2_prof.log; exit 1; }
f=$(find gpurun_out/vggwg2_prof -name "*kernel_stats.csv" | head -1)
python scripts/prof_summary.py $f 15 gpurun_out/vggwg2_kstats.csv > gpurun_out/vggwg2_ksum.txt; head -16 gpurun_out/vggwg2_ksum.txt
