#!/bin/bash
# End of round: full GPU suite, smoke, three ResNet-50 benches, launch counts, then one ResNet-50 kernel profile.
bash scripts/r5/gpu_final1.sh || exit 1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5/final_prof
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o rn50 -- python3 $R/bench.py --steps 3 --warmup 2 > $O/prof.log 2>&1 || exit 1
cd $R
python3 scripts/r5/trace_busy.py $(find $O/prof -name '*kernel_trace.csv') 60 > $O/resnet50_busy.txt || exit 1
find $O/prof -type f ! -name '*kernel_stats.csv' -delete
