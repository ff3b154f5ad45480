#!/bin/bash
# Kernel iteration on the 1-GPU box: GEMM/conv numerics tests, per-layer conv table, the headline
# bench, then the 3x3-conv PMC passes.  Stops at the first failing step.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/iter; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_kernels.py tests/test_gpu_hypothesis.py} > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python scripts/bench_resnet_layers.py > $O/layers.json 2> $O/layers.err || { tail $O/layers.err; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
tail -1 $O/bench.log
[ "${PMC:-1}" = 1 ] && bash scripts/pmc_conv.sh
exit 0
