#!/bin/bash
# End-of-round evidence at HEAD: full GPU suite + smoke, ResNet-50 bench x3, ResNet-50 kernel profile.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r4/final; mkdir -p $O
export TMPDIR=/tmp
( while true; do sleep 50; echo "[hb] $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -2 || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python bench.py 2>/dev/null > $O/b.json || exit 1
  cut -c1-150 $O/b.json | tee -a $O/bench.txt
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 $R/bench.py --steps 5 --warmup 2 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python3 $R/scripts/prof_summary.py "$f" 7 $O/resnet50_kernel_stats.csv | head -3
find $O/prof -name "*kernel_trace.csv" -delete
