#!/bin/bash
# GEMM routing knobs re-checked after the whole-wave statistics atomics (interleaved, ResNet-50 bench):
# tile fill rule, split-K rounds, gathered-wgrad rounds, raster group.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r4/knob_ab; mkdir -p $O
for i in 1 2; do
  for v in "DDL_X=0" "DDL_TILE_FILL=1" "DDL_TILE_FILL=4" "DDL_SPLIT_ROUNDS=4" "DDL_WGRAD_ROUNDS=2" "DDL_GEMM_GROUP_M=4" "DDL_GEMM_GROUP_M=16"; do
    env $v timeout -k 10 200 python bench.py --steps 20 --warmup 5 2>/dev/null > $O/b.json || exit 1
    echo "$v $(cut -c1-130 $O/b.json)" | tee -a $O/bench.txt
  done
done
