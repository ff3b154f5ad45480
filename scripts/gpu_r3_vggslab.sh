#!/bin/bash
# VGG-16 halo weight gradients: partial slabs + reduce (default) vs fp32 atomics, kernel time per step
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in 1 0; do
  ( cd /tmp && DDL_WGRAD3X3_SLAB=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/vggslab_$v -- python3 $R/bench.py --model vgg16 --steps 10 --warmup 5 > $R/gpurun_out/vggslab_$v.log 2>&1 ) || { echo "rocprof failed"; tail -20 gpurun_out/vggslab_$v.log; exit 1; }
  f=$(find gpurun_out/vggslab_$v -name "*kernel_stats.csv" | head -1)
  python scripts/prof_summary.py $f 15 gpurun_out/vggslab_kstats_$v.csv > gpurun_out/vggslab_ksum_$v.txt
  echo "slab=$v"; head -1 gpurun_out/vggslab_ksum_$v.txt; grep -E "wgrad" gpurun_out/vggslab_ksum_$v.txt
done
