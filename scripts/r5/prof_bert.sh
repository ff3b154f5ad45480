#!/bin/bash
# BERT-base MLM step: bench x2 + rocprofv3 kernel statistics (3 timed + 2 warmup steps) + busy summary.
export TMPDIR=/tmp
O=gpurun_out/r5/bert
mkdir -p $O
for i in 1 2; do timeout -k 10 300 python bench.py --model bert --steps 10 --warmup 3 > $O/bench_$i.log 2>&1 || exit 1; tail -1 $O/bench_$i.log | cut -c1-140; done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bert -- python bench.py --model bert --steps 3 --warmup 2 > $O/prof.log 2>&1 || exit 1
python scripts/r5/trace_busy.py $(find $O/prof -name '*kernel_trace.csv') 40 > $O/busy.txt
find $O/prof -type f ! -name '*stats.csv' -delete
