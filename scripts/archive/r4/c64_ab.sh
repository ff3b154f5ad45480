#!/bin/bash
# 64-channel 3x3 convs (ResNet-50 stage 1) on the halo kernel (DDL_CONV3X3_C64=1) or the resident-filter ping-pong
# kernel (DDL_CONV3X3_C64PP=1) vs the implicit GEMM (default), after the whole-wave statistics atomics; interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r4/c64; mkdir -p $O
for i in 1 2; do
  for v in "DDL_X=0" "DDL_CONV3X3_C64=1" "DDL_CONV3X3_C64PP=1"; do
    env $v timeout -k 10 200 python bench.py --steps 20 --warmup 5 2>/dev/null > $O/b.json || exit 1
    echo "$v $(cut -c1-130 $O/b.json)" | tee -a $O/bench.txt
  done
done
