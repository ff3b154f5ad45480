#!/bin/bash
# A/B of the BN streaming-sweep grid cap (DDL_BN_GRID 2048 / 4096 / 8192) and rows in flight (DDL_BN_ROWS 4),
# interleaved, ResNet-50 bench.
set -o pipefail
BN_GRID_SET=${BN_GRID_SET:-"DDL_BN_GRID=4096 DDL_BN_GRID=2048 DDL_BN_GRID=8192 DDL_BN_GRID=16384"}
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r4/bn_grid; mkdir -p $O
for i in 1 2; do
  for v in $BN_GRID_SET; do
    env $v timeout -k 10 200 python bench.py --steps 20 --warmup 5 2>/dev/null > $O/b.json || exit 1
    echo "$v $(cut -c1-140 $O/b.json)" | tee -a $O/bench.txt
  done
done
