#!/bin/bash
# End-of-round 1/2: full GPU suite, smoke, three ResNet-50 benches, steady-state launch counts.
export TMPDIR=/tmp
O=gpurun_out/r5/final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py > $O/bench_resnet50_$i.log 2>&1 || { tail -20 $O/bench_resnet50_$i.log; exit 1; }
  tail -1 $O/bench_resnet50_$i.log | cut -c1-150
done
MODELS="resnet50 vgg16" bash scripts/r5/launch_count.sh || exit 1
