#!/bin/bash
# Kernel trace of the timed (graph-replayed) ResNet-50 steps and their idle gaps (scripts/r6/trace_gaps.py).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6/gaps
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/rn50 -o rn50 -- python3 $R/bench.py --steps 8 --warmup 3 > $O/rn50.log 2>&1 || exit 1
python3 $R/scripts/r6/trace_gaps.py $(find $O/rn50 -name '*kernel_trace.csv') 5 > $O/rn50_gaps.txt || exit 1
find $O -type f -name '*kernel_trace.csv' -delete
