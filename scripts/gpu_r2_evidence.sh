#!/bin/bash
# Round-2 evidence: full GPU test suite, smoke, headline bench, per-layer conv table and kernel
# profiles of ResNet-50 / VGG-16 / BERT-base (summaries are copied into profiles/r2 by hand).
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/ev; mkdir -p $O
R=$(pwd)
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || exit 1
tail -1 $O/bench_default.log
timeout -k 10 300 python scripts/bench_resnet_layers.py > $O/layers.json 2> /dev/null || exit 1
for m in resnet50 vgg16 bert; do
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ev/prof_$m -- python3 $R/bench.py --model $m --steps 5 --warmup 2 > $R/gpurun_out/ev/prof_$m.log 2>&1 || { echo "prof $m failed"; exit 1; }
  cd $R
  echo "prof $m ok"
done
