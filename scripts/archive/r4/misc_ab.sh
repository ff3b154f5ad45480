#!/bin/bash
# Cheap knob A/B at HEAD (interleaved, ResNet-50): BN sweep rows per lane (DDL_BN_ROWS 2 / 4, uncapped grids) and
# the stem BN reduce's workgroups (DDL_STEM_PARTIALS 2048 / 4096 / 8192).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r4/misc_ab; mkdir -p $O
for i in 1 2; do
  for v in "DDL_X=0" "DDL_BN_ROWS=4" "DDL_STEM_PARTIALS=4096" "DDL_STEM_PARTIALS=8192"; do
    env $v timeout -k 10 200 python bench.py --steps 20 --warmup 5 2>/dev/null > $O/b.json || exit 1
    echo "$v $(cut -c1-130 $O/b.json)" | tee -a $O/bench.txt
  done
done
