#!/bin/bash
# Kernel trace of 3 ResNet-50 steps: per-call BN sweep durations (bn_apply / bn_bwd_dx by grid) for a
# per-layer bandwidth table (scripts/r4/bn_trace_table.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4/bn_trace; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -- python3 $R/bench.py --steps 3 --warmup 2 > $O/run.log 2>&1 || exit 1
f=$(find $O/tr -name "*kernel_trace.csv" | head -1)
python3 $R/scripts/r4/bn_trace_table.py "$f" > $O/table.txt && cat $O/table.txt
find $O/tr -name "*kernel_trace.csv" -delete
