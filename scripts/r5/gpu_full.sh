#!/bin/bash
# Full GPU suite + smoke + 1-GPU bench at HEAD, then steady-state launch counts.
export TMPDIR=/tmp
O=gpurun_out/r5/full
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
MODELS="resnet50 vgg16" bash scripts/r5/launch_count.sh || exit 1
