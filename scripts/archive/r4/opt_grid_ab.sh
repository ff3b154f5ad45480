#!/bin/bash
# Uncapped optimizer / misc / slab-reduce grids (default now) vs the old caps, interleaved: BERT-base and ResNet-50.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r4/opt_grid; mkdir -p $O
for i in 1 2; do
  for m in bert resnet50; do
    for v in "DDL_OPT_GRID=4096 DDL_MISC_GRID=4096" "DDL_X=0" "DDL_LN_FWD_BLOCKS=65536"; do
      env $v timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 2>/dev/null > $O/b.json || exit 1
      echo "$m $v $(cut -c1-130 $O/b.json)" | tee -a $O/bench.txt
    done
  done
done
