#!/bin/bash
# BERT-base kernel profile at HEAD (3 timed + 2 warmup steps), summarised by scripts/r5/trace_busy.py.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6/prof2
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bert -o bert -- python3 $R/bench.py --model bert --steps 3 --warmup 2 > $O/bert.log 2>&1 || exit 1
python3 $R/scripts/r5/trace_busy.py $(find $O/bert -name '*kernel_trace.csv') 45 > $O/bert_busy.txt || exit 1
find $O -type f -name '*kernel_trace.csv' -delete
