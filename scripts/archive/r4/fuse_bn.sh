#!/bin/bash
# BN-backward reduce fusions (shortcut BN in bn3's dx sweep, streaming mode-2 reduce, residual / strided-class
# BNR epilogues): tests, probe of the remaining reduce sweeps, bench x3, ResNet-50 kernel profile.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r4/fuse_bn; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread \
  -k "bnr or bn_bwd or bottleneck or fused_bn or resnet or strided or stem" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/probe_bn_calls.py > $O/probe.txt 2>&1 || exit 1
head -3 $O/probe.txt
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 2>/dev/null | tee -a $O/bench.jsonl | cut -c1-200 || exit 1
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 $R/bench.py --steps 5 --warmup 2 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python3 $R/scripts/prof_summary.py "$f" 7 $O/resnet50_kernel_stats.csv | head -20
find $O/prof -name "*kernel_trace.csv" -delete
