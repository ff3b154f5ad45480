#!/bin/bash
# Round 3: rocprofv3 kernel stats of the ResNet-50 bench under two values of one env knob.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
VAR=${AB_VAR:-DDL_NORM_ON_LOAD}
export TMPDIR=/tmp
VALS=${AB_VALUES:-1 0}
for v in $VALS; do
  ( cd /tmp && export $VAR=$v && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_${VAR}_$v -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 ${BENCH_ARGS:-} > $GRAFT_REPO_ROOT/gpurun_out/prof_${VAR}_$v.log 2>&1 ) || { echo "rocprof $VAR=$v failed"; tail -20 gpurun_out/prof_${VAR}_$v.log; exit 1; }
  f=$(find gpurun_out/prof_${VAR}_$v -name "*kernel_stats.csv" | head -1)
  python scripts/prof_summary.py $f 5 gpurun_out/kstats_${VAR}_$v.csv | head -3
done
