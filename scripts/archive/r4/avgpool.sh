#!/bin/bash
# avgpool forward unroll: pooling tests, then the final suite (tests + smoke + bench + profile).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "avgpool or pool" > gpurun_out/r4/avgpool_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r4/avgpool_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/r4/final.sh
