#!/bin/bash
# Full GPU suite + smoke + 3 ResNet-50 benches (the driver's default command) on one box.
set -o pipefail
mkdir -p gpurun_out/r6/suite
O=gpurun_out/r6/suite
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py > $O/bench_$i.json 2> $O/bench_$i.err || exit 1
done
cat $O/bench_*.json | cut -c1-200
