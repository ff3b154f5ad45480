#!/bin/bash
# ResNet-50 bench at HEAD, then VGG-16 bench x3 + rocprofv3 kernel stats of the VGG-16 step
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/vp_resnet.log 2>&1 || { tail -20 gpurun_out/vp_resnet.log; exit 1; }
grep '^{' gpurun_out/vp_resnet.log | cut -c1-200
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --model vgg16 --steps 50 --warmup 10 > gpurun_out/vp_vgg.log 2>&1 || { tail -20 gpurun_out/vp_vgg.log; exit 1; }
  grep '^{' gpurun_out/vp_vgg.log | cut -c1-200
done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/vgg_prof -- python3 $GRAFT_REPO_ROOT/bench.py --model vgg16 --steps 10 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/vgg_prof.log 2>&1 ) || { echo "rocprof failed"; tail -20 gpurun_out/vgg_prof.log; exit 1; }
f=$(find gpurun_out/vgg_prof -name "*kernel_stats.csv" | head -1)
python scripts/prof_summary.py $f 15 gpurun_out/vgg_kstats.csv | head -40
