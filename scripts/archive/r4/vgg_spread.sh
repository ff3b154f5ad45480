#!/bin/bash
# VGG-16 run-to-run spread: 4 bench runs, then two kernel traces of the bench (busy vs idle per step).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4/vgg
export TMPDIR=/tmp
for i in 1 2; do
  for g in 0 1; do
    timeout -k 10 200 python bench.py --model vgg16 --steps 30 --warmup 5 --graph $g 2>/dev/null | grep '^{' | sed "s/^/graph=$g /" >> gpurun_out/r4/vgg/bench_runs.txt || exit 1
  done
done
python -c "
import json
for l in open('gpurun_out/r4/vgg/bench_runs.txt'):
    t, js = l.split(' ', 1); d = json.loads(js); print(t, round(d['value']), d['ms_per_step'])"
for i in 1 2; do
  ( cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4/vgg/trace$i -- python3 $GRAFT_REPO_ROOT/bench.py --model vgg16 --steps 30 --warmup 5 --graph $((i - 1)) > $GRAFT_REPO_ROOT/gpurun_out/r4/vgg/trace$i.log 2>&1 ) || exit 1
  grep '^{' gpurun_out/r4/vgg/trace$i.log | head -1
  python scripts/r4/trace_gaps.py $(find gpurun_out/r4/vgg/trace$i -name "*kernel_trace.csv" | head -1) > gpurun_out/r4/vgg/gaps$i.txt
  tail -1 gpurun_out/r4/vgg/gaps$i.txt
done
