#!/bin/bash
# Round 3: DataFrame-fed ResNet-50 vs the plain bench at HEAD, one box, interleaved.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out/dataframe_vs_plain_r3.jsonl
: > $OUT
for r in 1 2; do
  for v in plain resident stream pool; do
    case $v in
      plain) a="";;
      resident) a="--via-dataframe --ingest resident";;
      stream) a="--via-dataframe --ingest stream";;
      pool) a="--via-dataframe --ingest resident --executor-pool";;
    esac
    timeout -k 10 400 python bench.py --steps 20 --warmup 5 $a > gpurun_out/df_tmp.log 2>&1 || { echo "$v failed"; tail -30 gpurun_out/df_tmp.log; exit 1; }
    line=$(grep '^{' gpurun_out/df_tmp.log | tail -1)
    echo "{\"round\": $r, \"variant\": \"$v\", \"bench\": $line}" >> $OUT
    echo "r$r $v $(echo $line | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
  done
done
