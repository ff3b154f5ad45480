#!/bin/bash
# Uncapped sweep grids (default now) vs the old caps (DDL_BN_GRID=4096 DDL_POOL_GRID=8192) vs pool-only old cap,
# interleaved, ResNet-50; then BN / pool / GEMM tests.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r4/pool_grid; mkdir -p $O
for i in 1 2; do
  for v in "DDL_BN_GRID=4096 DDL_POOL_GRID=8192" "DDL_POOL_GRID=8192" "DDL_X=0"; do
    env $v timeout -k 10 200 python bench.py --steps 20 --warmup 5 2>/dev/null > $O/b.json || exit 1
    echo "$v $(cut -c1-140 $O/b.json)" | tee -a $O/bench.txt
  done
done
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_layers.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; exit $rc
