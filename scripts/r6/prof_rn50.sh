#!/bin/bash
# ResNet-50 kernel profile at HEAD (5 timed + 3 warmup steps), summarised by scripts/r5/trace_busy.py.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6/prof2
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rn50 -o rn50 -- python3 $R/bench.py --steps 5 --warmup 3 > $O/rn50.log 2>&1 || exit 1
python3 $R/scripts/r5/trace_busy.py $(find $O/rn50 -name '*kernel_trace.csv') 45 > $O/rn50_busy.txt || exit 1
find $O -type f -name '*kernel_trace.csv' -delete
