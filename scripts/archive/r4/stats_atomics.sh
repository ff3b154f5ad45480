#!/bin/bash
# Whole-wave statistics atomics (butterfly reduce-scatter) in the GEMM epilogues: GEMM / conv / BN tests,
# ResNet-50 bench x3, kernel profile.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r4/stats_atomics; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_gemm256.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 2>/dev/null > $O/b.json || exit 1
  cut -c1-150 $O/b.json | tee -a $O/bench.txt
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 $R/bench.py --steps 5 --warmup 2 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python3 $R/scripts/prof_summary.py "$f" 7 $O/resnet50_kernel_stats.csv | head -3
find $O/prof -name "*kernel_trace.csv" -delete
