#!/bin/bash
# Round-4 BN fusions, second pass: tests, A/B of the strided-class BNR (DDL_STRIDED_BNR 0 / 1, interleaved),
# kernel profile at the default.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r4/fuse_bn2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread \
  -k "bnr or bn_bwd or bottleneck or fused_bn or resnet or strided or stem" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for v in 0 1; do
    DDL_STRIDED_BNR=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 2>/dev/null > $O/b.json || exit 1
    echo "strided_bnr=$v $(cut -c1-150 $O/b.json)" | tee -a $O/bench.txt
  done
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 $R/bench.py --steps 5 --warmup 2 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python3 $R/scripts/prof_summary.py "$f" 7 $O/resnet50_kernel_stats.csv | head -3
find $O/prof -name "*kernel_trace.csv" -delete
