#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_layers.py -k "derived" > gpurun_out/r5/t_derived.log 2>&1 || { echo TESTS FAILED; grep -E "Error|^E " gpurun_out/r5/t_derived.log | head -30; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/r5/t_derived.log
ROUNDS=3 TAG=ab_derived bash scripts/r5/ab.sh || exit 1
for i in 1 2 3; do timeout -k 10 200 python bench.py --model vgg16 --steps 50 --warmup 10 > gpurun_out/r5/vggd_$i.log 2>&1 || exit 1; tail -1 gpurun_out/r5/vggd_$i.log | cut -c1-130; done
