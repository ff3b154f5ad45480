#!/bin/bash
# VGG-16 spread (graph 0/1 runs + two kernel traces with per-step busy / idle), kernel profiles of the three
# benches at HEAD, and a kernel profile of BERT-base in deterministic mode.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4/prof
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "[batch7] fatal rc=$1 in $2"; exit $1;; esac; }
bash scripts/r4/vgg_spread.sh; rc=$?; echo "[batch7] vgg_spread rc=$rc"; fatal $rc vgg
bash scripts/r4/prof.sh; rc=$?; echo "[batch7] prof rc=$rc"; fatal $rc prof
R=$PWD
( cd /tmp && DDL_DETERMINISTIC=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r4/prof/bert_det -- python3 $R/bench.py --model bert --steps 5 --warmup 2 > $R/gpurun_out/r4/prof/bert_det.log 2>&1 )
rc=$?; echo "[batch7] bert det prof rc=$rc"; fatal $rc bert_det
f=$(find gpurun_out/r4/prof/bert_det -name "*kernel_stats.csv" | head -1)
python3 scripts/prof_summary.py "$f" 7 gpurun_out/r4/prof/bert_det_kernel_stats.csv | head -16
find gpurun_out/r4/prof/bert_det -name "*kernel_trace.csv" -delete
exit 0
