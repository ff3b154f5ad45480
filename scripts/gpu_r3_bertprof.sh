#!/bin/bash
# BERT-base kernel profile at HEAD
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/bert_prof -- python3 $R/bench.py --model bert --steps 5 --warmup 2 > $R/gpurun_out/bert_prof.log 2>&1 ) || { echo "rocprof failed"; tail $R/gpurun_out/bert_prof.log; exit 1; }
f=$(find gpurun_out/bert_prof -name "*kernel_stats.csv" | head -1)
python scripts/prof_summary.py $f 7 gpurun_out/bert_kstats.csv | head -40
