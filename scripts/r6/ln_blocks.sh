#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6
out=gpurun_out/r6/ln_blocks.txt
: > $out
for b in 512 768 1024 1536; do
  DDL_LN_BWD_BLOCKS=$b timeout -k 10 100 python -u scripts/r6/bench_ln_bwd.py 2>/dev/null | sed "s/^/blocks=$b /" >> $out || exit 1
done
cat $out
