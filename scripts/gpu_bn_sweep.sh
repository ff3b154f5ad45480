#!/bin/bash
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/bn; mkdir -p $O
for p in 512 1024 2048 4096; do
  echo "partials=$p"
  DDL_BN_PARTIALS=$p timeout -k 10 120 python scripts/bench_bn.py > $O/bn_$p.log 2>&1 || { tail $O/bn_$p.log; exit 1; }
  cat $O/bn_$p.log
done
