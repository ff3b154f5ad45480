#!/bin/bash
# Quick kernel iteration: conv/GEMM numerics, per-layer table, headline bench (optionally with an
# extra env assignment list in $VARIANT applied to a second layer table + bench).
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/quick; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_hypothesis.py ${EXTRA_TESTS:-} > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python scripts/bench_resnet_layers.py > $O/layers.json 2> $O/layers.err || { tail $O/layers.err; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-140
if [ -n "${VARIANT:-}" ]; then
  env $VARIANT timeout -k 10 300 python scripts/bench_resnet_layers.py > $O/layers_v.json 2> $O/layers_v.err || exit 1
  env $VARIANT timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_v.log 2>&1 || exit 1
  tail -1 $O/bench_v.log | cut -c1-140
fi
exit 0
