#!/bin/bash
# Fused BN forward finalize (GemmParams.fin_*): tests, then A/B (DDL_FUSE_BN_FINALIZE 0 / 1) interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r4/fin; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread \
  -k "fused_bn_finalize or bottleneck or resnet or bn_" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for v in 0 1; do
    DDL_FUSE_BN_FINALIZE=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 2>/dev/null > $O/b.json || exit 1
    echo "fuse_finalize=$v $(cut -c1-140 $O/b.json)" | tee -a $O/bench.txt
  done
done
