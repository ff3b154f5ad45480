#!/bin/bash
# Weight-gradient LDS ring depth: numerics of the conv / GEMM tests and the per-layer table at
# DDL_WGRAD_STAGES = 3 and 4 (default 1 = single-stage kernel).
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/ring; mkdir -p $O
export TMPDIR=/tmp
for st in 3 4; do
  DDL_WGRAD_STAGES=$st timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_kernels.py tests/test_gpu_hypothesis.py -k "gemm or conv or resnet or bottleneck" > $O/tests_st$st.log 2>&1 \
    || { tail -30 $O/tests_st$st.log; exit 1; }
  tail -1 $O/tests_st$st.log
  DDL_WGRAD_STAGES=$st timeout -k 10 300 python scripts/bench_resnet_layers.py > $O/layers_st$st.json 2> $O/layers_st$st.err || { tail $O/layers_st$st.err; exit 1; }
done
timeout -k 10 300 python scripts/bench_resnet_layers.py > $O/layers_st1.json 2> $O/layers_st1.err || exit 1
DDL_WGRAD_STAGES=3 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_st3.log 2>&1 || { tail $O/bench_st3.log; exit 1; }
tail -1 $O/bench_st3.log | cut -c1-150
DDL_WGRAD_STAGES=4 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_st4.log 2>&1 || { tail $O/bench_st4.log; exit 1; }
tail -1 $O/bench_st4.log | cut -c1-150
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_st1.log 2>&1 || exit 1
tail -1 $O/bench_st1.log | cut -c1-150
