#!/bin/bash
# A/B: BN-reducing data-gradients on the streaming kernel (max panels 64 = always) vs the LDS-DMA BNR GEMM
# beyond 4 / 2 panels (DDL_BNR_STREAM_MAX_PANELS), interleaved, ResNet-50 bench.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r4/bnr_panels; mkdir -p $O
for i in 1 2; do
  for v in 64 4 2; do
    DDL_BNR_STREAM_MAX_PANELS=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 2>/dev/null > $O/b.json || exit 1
    echo "max_panels=$v $(cut -c1-150 $O/b.json)" | tee -a $O/bench.txt
  done
done
